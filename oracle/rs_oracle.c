/*
 * rs_oracle.c -- CPU oracle for the Reed-Solomon GF(2^16) hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as a checker /
 * reported baseline.  The product (librs_mi355x.so) never links or calls it.
 *
 * A plain-C restatement of the semantics of AndersTrier/reed-solomon-simd
 * v3.1.0 (Rust, mounted read-only at /root/reference; it cannot be compiled in
 * this image -- no Rust toolchain).  Written from the semantics, radix-2
 * "Naive engine" style; the parity anchor is the reference's own SHA-256
 * golden vectors (src/test_util.rs:575-850), checked by tests/test_oracle_golden.py.
 *
 * Reference anchors (paths relative to /root/reference):
 *   GF constants ............ src/engine.rs:199-221
 *   exp/log (Cantor basis) .. src/engine/tables.rs:184-221
 *   log_walsh ............... src/engine/tables.rs:223-233
 *   skew (twiddle logs) ..... src/engine/tables.rs:285-324
 *   scalar mul .............. src/engine/tables.rs:172-178
 *   add_mod / sub_mod ....... src/engine/utils.rs:59-69
 *   eval_poly / fwht ........ src/engine/utils.rs:20-31, src/engine/fwht.rs:9-55
 *   formal_derivative ....... src/engine/utils.rs:99-104
 *   Naive fft / ifft / mul .. src/engine/engine_naive.rs:43-146
 *   shard layout / tail ..... src/engine/shards.rs:38-74
 *   HighRate enc/dec ........ src/rate/rate_high.rs:44-87, 172-254, 135-141, 308-312
 *   LowRate enc/dec ......... src/rate/rate_low.rs:44-87, 172-254, 135-141, 308-312
 *   rate selection .......... src/rate/rate_default.rs:15-64
 *   test RNG (ChaCha8) ...... src/test_util.rs:76-87 (rand_chacha 0.3 / rand_core 0.6 fill_bytes)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GF_BITS 16
#define GF_ORDER 65536u
#define GF_MOD 65535u
#define GF_POLY 0x1002Du

typedef uint16_t gf;

static const gf kCantor[GF_BITS] = {
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

static gf g_exp[GF_ORDER];
static gf g_log[GF_ORDER];
static gf g_skew[GF_MOD];
static gf g_log_walsh[GF_ORDER];
static int g_ready = 0;

/* ------------------------------------------------------------------ */
/* mod-65535 arithmetic (utils.rs:59-69)                               */

static inline gf add_mod(gf a, gf b) {
    uint32_t s = (uint32_t)a + b;
    return (gf)(s + (s >> 16));
}
static inline gf sub_mod(gf a, gf b) {
    uint32_t d = (uint32_t)a - (uint32_t)b;
    return (gf)(d + (d >> 16));
}
/* x * exp(log_m); 0 stays 0 (tables.rs:172-178) */
static inline gf gf_mul_log(gf x, gf log_m) {
    return x ? g_exp[add_mod(g_log[x], log_m)] : 0;
}

/* Walsh-Hadamard transform over Z/65535, radix-2 DIT (fwht.rs). */
static void fwht(gf *v, uint32_t n) {
    for (uint32_t h = 1; h < n; h <<= 1)
        for (uint32_t base = 0; base < n; base += 2 * h)
            for (uint32_t i = base; i < base + h; i++) {
                gf a = v[i], b = v[i + h];
                v[i] = add_mod(a, b);
                v[i + h] = sub_mod(a, b);
            }
}

void orc_init(void) {
    if (g_ready) return;
    /* LFSR pass: polynomial-basis element -> discrete log. */
    static _Thread_local gf plog[GF_ORDER];
    uint32_t st = 1;
    for (uint32_t k = 0; k < GF_MOD; k++) {
        plog[st] = (gf)k;
        st <<= 1;
        if (st >= GF_ORDER) st ^= GF_POLY;
    }
    plog[0] = GF_MOD;
    /* Cantor coordinates -> polynomial element -> log. */
    static _Thread_local gf poly[GF_ORDER];
    poly[0] = 0;
    for (int b = 0; b < GF_BITS; b++) {
        uint32_t w = 1u << b;
        for (uint32_t j = 0; j < w; j++) poly[w + j] = poly[j] ^ kCantor[b];
    }
    for (uint32_t j = 0; j < GF_ORDER; j++) g_log[j] = plog[poly[j]];
    for (uint32_t j = 0; j < GF_ORDER; j++) g_exp[g_log[j]] = (gf)j;
    g_exp[GF_MOD] = g_exp[0];

    /* Twiddle (skew) table, tables.rs:285-324, restated. */
    gf raw[GF_MOD];
    memset(raw, 0, sizeof raw);
    gf basis[GF_BITS - 1];
    for (int b = 1; b < GF_BITS; b++) basis[b - 1] = (gf)(1u << b);
    for (int m = 0; m < GF_BITS - 1; m++) {
        uint32_t step = 1u << (m + 1);
        raw[(1u << m) - 1] = 0;
        for (int i = m; i < GF_BITS - 1; i++) {
            uint32_t s = 1u << (i + 1);
            for (uint32_t j = (1u << m) - 1; j < s; j += step) raw[j + s] = raw[j] ^ basis[i];
        }
        basis[m] = (gf)(GF_MOD - g_log[gf_mul_log(basis[m], g_log[basis[m] ^ 1])]);
        for (int i = m + 1; i < GF_BITS - 1; i++) {
            gf e = add_mod(g_log[basis[i] ^ 1], basis[m]);
            basis[i] = gf_mul_log(basis[i], e);
        }
    }
    for (uint32_t i = 0; i < GF_MOD; i++) g_skew[i] = g_log[raw[i]];

    /* LogWalsh: FWHT of log[] with log[0] := 0 (tables.rs:223-233). */
    memcpy(g_log_walsh, g_log, sizeof g_log_walsh);
    g_log_walsh[0] = 0;
    fwht(g_log_walsh, GF_ORDER);
    g_ready = 1;
}

const uint16_t *orc_exp_table(void) { orc_init(); return g_exp; }
const uint16_t *orc_log_table(void) { orc_init(); return g_log; }
const uint16_t *orc_skew_table(void) { orc_init(); return g_skew; }
const uint16_t *orc_log_walsh_table(void) { orc_init(); return g_log_walsh; }

uint16_t orc_gf_mul(uint16_t x, uint16_t log_m) { orc_init(); return gf_mul_log(x, log_m); }

/* ------------------------------------------------------------------ */
/* Engine ops over a shard matrix: `rows` rows of `blocks` 64-byte blocks, */
/* each block = 32 lo bytes then 32 hi bytes (algorithm.md "Shard").      */

static inline uint8_t *row_ptr(uint8_t *d, size_t blocks, size_t r) { return d + r * blocks * 64; }

static void xor_row(uint8_t *dst, const uint8_t *src, size_t blocks) {
    for (size_t i = 0; i < blocks * 64; i++) dst[i] ^= src[i];
}

/* dst ^= src * exp(log_m) */
static void muladd_row(uint8_t *dst, const uint8_t *src, size_t blocks, gf log_m) {
    for (size_t b = 0; b < blocks; b++) {
        const uint8_t *s = src + 64 * b;
        uint8_t *t = dst + 64 * b;
        for (int e = 0; e < 32; e++) {
            gf p = gf_mul_log((gf)(s[e] | (s[e + 32] << 8)), log_m);
            t[e] ^= (uint8_t)p;
            t[e + 32] ^= (uint8_t)(p >> 8);
        }
    }
}

void orc_mul(uint8_t *rows, size_t blocks, uint16_t log_m) {
    orc_init();
    for (size_t b = 0; b < blocks; b++) {
        uint8_t *t = rows + 64 * b;
        for (int e = 0; e < 32; e++) {
            gf p = gf_mul_log((gf)(t[e] | (t[e + 32] << 8)), log_m);
            t[e] = (uint8_t)p;
            t[e + 32] = (uint8_t)(p >> 8);
        }
    }
}

/* Decimation-in-time FFT on rows [pos, pos+size) (engine_naive.rs:43-73).
 * Twiddle of group r at distance d: skew[r + d + skew_delta - 1];
 * 65535 means "no multiply" (butterfly degenerates to XOR). */
void orc_fft(uint8_t *data, size_t blocks, size_t pos, size_t size, size_t truncated, size_t skew_delta) {
    orc_init();
    for (size_t d = size / 2; d > 0; d /= 2)
        for (size_t r = 0; r < truncated; r += 2 * d) {
            gf lm = g_skew[r + d + skew_delta - 1];
            for (size_t i = r; i < r + d; i++) {
                uint8_t *a = row_ptr(data, blocks, pos + i), *b = row_ptr(data, blocks, pos + i + d);
                if (lm != GF_MOD) muladd_row(a, b, blocks, lm);
                xor_row(b, a, blocks);
            }
        }
}

/* Inverse transform (engine_naive.rs:75-105). */
void orc_ifft(uint8_t *data, size_t blocks, size_t pos, size_t size, size_t truncated, size_t skew_delta) {
    orc_init();
    for (size_t d = 1; d < size; d *= 2)
        for (size_t r = 0; r < truncated; r += 2 * d) {
            gf lm = g_skew[r + d + skew_delta - 1];
            for (size_t i = r; i < r + d; i++) {
                uint8_t *a = row_ptr(data, blocks, pos + i), *b = row_ptr(data, blocks, pos + i + d);
                xor_row(b, a, blocks);
                if (lm != GF_MOD) muladd_row(a, b, blocks, lm);
            }
        }
}

/* utils.rs:99-104, sequential definition. */
void orc_formal_derivative(uint8_t *data, size_t blocks, size_t rows) {
    for (size_t i = 1; i < rows; i++) {
        size_t w = i & (~i + 1);
        for (size_t k = 0; k < w; k++)
            xor_row(row_ptr(data, blocks, i - w + k), row_ptr(data, blocks, i + k), blocks);
    }
}

/* utils.rs:20-31 */
void orc_eval_poly(uint16_t *er, size_t truncated) {
    orc_init();
    (void)truncated; /* truncated FWHT == full FWHT for an input that is zero past `truncated` */
    fwht(er, GF_ORDER);
    for (uint32_t i = 0; i < GF_ORDER; i++) {
        uint32_t p = (uint32_t)er[i] * g_log_walsh[i];
        er[i] = add_mod((gf)p, (gf)(p >> 16));
    }
    fwht(er, GF_ORDER);
}

/* Engine selection for the rate layer: 0 = radix-2 restatement above
 * (the oracle), 1 = AVX2 restatement in avx2_port.c (the CPU baseline). */
typedef void (*xform_fn)(uint8_t *, size_t, size_t, size_t, size_t, size_t);
typedef void (*mul_fn)(uint8_t *, size_t, uint16_t);
void avx2_fft(uint8_t *, size_t, size_t, size_t, size_t, size_t);
void avx2_ifft(uint8_t *, size_t, size_t, size_t, size_t, size_t);
void avx2_mul(uint8_t *, size_t, uint16_t);
int avx2_available(void);
static xform_fn E_fft = orc_fft, E_ifft = orc_ifft;
static mul_fn E_mul = orc_mul;

/* returns 0 on success, -1 if the engine is unavailable on this CPU */
int orc_select_engine(int which) {
    orc_init();
    if (which == 1) {
        if (!avx2_available()) return -1;
        E_fft = avx2_fft; E_ifft = avx2_ifft; E_mul = avx2_mul;
    } else {
        E_fft = orc_fft; E_ifft = orc_ifft; E_mul = orc_mul;
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Shard layout (shards.rs:38-74)                                      */

static void insert_shard(uint8_t *work, size_t blocks, size_t row, const uint8_t *src, size_t S) {
    uint8_t *dst = row_ptr(work, blocks, row);
    size_t whole = S / 64, tail = S % 64;
    memcpy(dst, src, whole * 64);
    if (tail) {
        uint8_t *blk = dst + whole * 64;
        memcpy(blk, src + whole * 64, tail / 2);
        memcpy(blk + 32, src + whole * 64 + tail / 2, tail / 2);
    }
}
static void extract_shard(const uint8_t *work, size_t blocks, size_t row, uint8_t *out, size_t S) {
    const uint8_t *src = work + row * blocks * 64;
    size_t whole = S / 64, tail = S % 64;
    memcpy(out, src, whole * 64);
    if (tail) {
        const uint8_t *blk = src + whole * 64;
        memcpy(out + whole * 64, blk, tail / 2);
        memcpy(out + whole * 64 + tail / 2, blk + 32, tail / 2);
    }
}

/* Work buffer re-used across calls, like the reference's EncoderWork /
 * DecoderWork (shards.rs:30-36 keeps its allocation). */
static _Thread_local uint8_t *g_work = NULL; /* per thread: bench.py times the CPU baseline on all cores */
static _Thread_local size_t g_work_cap = 0;
static uint8_t *work_buf(size_t bytes) {
    if (bytes > g_work_cap) {
        free(g_work);
        g_work = malloc(bytes);
        g_work_cap = bytes;
    }
    memset(g_work, 0, bytes);
    return g_work;
}

static size_t next_pow2(size_t x) { size_t p = 1; while (p < x) p <<= 1; return p; }
static size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

/* Error codes mirror include/rs_mi355x.h */
enum { E_OK = 0, E_UNSUPPORTED = 10, E_SHARD_SIZE = 6, E_NOT_ENOUGH = 7 };

static int high_supported(size_t N, size_t M) {
    return N > 0 && M > 0 && N < GF_ORDER && M < GF_ORDER && next_pow2(M) + N <= GF_ORDER;
}
static int low_supported(size_t N, size_t M) {
    return N > 0 && M > 0 && N < GF_ORDER && M < GF_ORDER && next_pow2(N) + M <= GF_ORDER;
}

/* rate_default.rs:15-64: 1 = high, 0 = low, -1 = unsupported */
int orc_use_high_rate(size_t N, size_t M) {
    if (N > GF_ORDER || M > GF_ORDER || N == 0 || M == 0) return -1;
    size_t pn = next_pow2(N), pm = next_pow2(M);
    size_t small = pn < pm ? pn : pm, large = N > M ? N : M;
    if (small + large > GF_ORDER) return -1;
    if (pn < pm) return 0;
    if (pn > pm) return 1;
    return N <= M ? 1 : 0;
}

static int resolve_rate(int rate, size_t N, size_t M, size_t S) {
    int high;
    if (rate == 1) high = 1;
    else if (rate == 2) high = 0;
    else {
        int u = orc_use_high_rate(N, M);
        if (u < 0) return -E_UNSUPPORTED;
        high = u;
    }
    if (high ? !high_supported(N, M) : !low_supported(N, M)) return -E_UNSUPPORTED;
    if (S == 0 || (S & 1)) return -E_SHARD_SIZE;
    return high;
}

/* rate: 0 = default (use_high_rate), 1 = HighRate, 2 = LowRate.
 * orig: N*S bytes, rec out: M*S bytes.  Returns 0 or an error code. */
int orc_encode(int rate, size_t N, size_t M, size_t S, const uint8_t *orig, uint8_t *rec) {
    orc_init();
    int high = resolve_rate(rate, N, M, S);
    if (high < 0) return -high;
    size_t blocks = (S + 63) / 64;
    if (high) {
        size_t n = next_pow2(M), rows = round_up(N, n);
        uint8_t *w = work_buf(rows * blocks * 64);
        for (size_t i = 0; i < N; i++) insert_shard(w, blocks, i, orig + i * S, S);
        /* rate_high.rs:44-87: chunk c transformed with skew_delta = c*n + n,
         * all chunks XOR-folded into chunk 0, then one FFT with skew_delta 0. */
        size_t first = N < n ? N : n;
        E_ifft(w, blocks, 0, n, first, n);
        for (size_t c0 = n; c0 < N; c0 += n) {
            size_t cnt = N - c0 < n ? N - c0 : n;
            E_ifft(w, blocks, c0, n, cnt, c0 + n);
            for (size_t r = 0; r < n; r++) xor_row(row_ptr(w, blocks, r), row_ptr(w, blocks, c0 + r), blocks);
        }
        E_fft(w, blocks, 0, n, M, 0);
        for (size_t i = 0; i < M; i++) extract_shard(w, blocks, i, rec + i * S, S);
    } else {
        size_t n = next_pow2(N), rows = round_up(M, n);
        uint8_t *w = work_buf(rows * blocks * 64);
        for (size_t i = 0; i < N; i++) insert_shard(w, blocks, i, orig + i * S, S);
        /* rate_low.rs:44-87: one IFFT (skew 0), replicated into every output
         * chunk, chunk c transformed with FFT skew_delta = c*n + n. */
        E_ifft(w, blocks, 0, n, N, 0);
        for (size_t c0 = n; c0 < M; c0 += n) memcpy(row_ptr(w, blocks, c0), w, n * blocks * 64);
        for (size_t c0 = 0; c0 < M; c0 += n) {
            size_t cnt = M - c0 < n ? M - c0 : n;
            E_fft(w, blocks, c0, n, cnt, c0 + n);
        }
        for (size_t i = 0; i < M; i++) extract_shard(w, blocks, i, rec + i * S, S);
    }
    return E_OK;
}

/* orig_present[i] / rec_present[i] != 0 mark provided shards.  Restored
 * originals (only those not present) are written to restored + i*S. */
int orc_decode(int rate, size_t N, size_t M, size_t S, const uint8_t *orig, const uint8_t *orig_present,
               const uint8_t *rec, const uint8_t *rec_present, uint8_t *restored) {
    orc_init();
    int high = resolve_rate(rate, N, M, S);
    if (high < 0) return -high;
    size_t have_o = 0, have_r = 0;
    for (size_t i = 0; i < N; i++) have_o += orig_present[i] != 0;
    for (size_t i = 0; i < M; i++) have_r += rec_present[i] != 0;
    if (have_o + have_r < N) return E_NOT_ENOUGH;
    if (have_o == N) return E_OK;

    size_t blocks = (S + 63) / 64;
    /* decoder_work.rs / rate_*.rs: recovery and original positions. */
    size_t chunk = high ? next_pow2(M) : next_pow2(N);
    size_t rec_base = high ? 0 : chunk, orig_base = high ? chunk : 0;
    size_t rows = next_pow2(chunk + (high ? N : M));
    uint8_t *w = work_buf(rows * blocks * 64);
    uint8_t *got = calloc(rows, 1);
    for (size_t i = 0; i < N; i++)
        if (orig_present[i]) { insert_shard(w, blocks, orig_base + i, orig + i * S, S); got[orig_base + i] = 1; }
    for (size_t i = 0; i < M; i++)
        if (rec_present[i]) { insert_shard(w, blocks, rec_base + i, rec + i * S, S); got[rec_base + i] = 1; }

    uint16_t *er = calloc(GF_ORDER, sizeof(uint16_t));
    size_t end;
    if (high) {
        end = chunk + N; /* rate_high.rs:186-204 */
        for (size_t i = 0; i < M; i++) er[i] = !got[i];
        for (size_t i = M; i < chunk; i++) er[i] = 1;
        for (size_t i = chunk; i < end; i++) er[i] = !got[i];
        orc_eval_poly(er, end);
    } else {
        end = chunk + M; /* rate_low.rs:186-204 */
        for (size_t i = 0; i < N; i++) er[i] = !got[i];
        for (size_t i = chunk; i < end; i++) er[i] = !got[i];
        for (size_t i = end; i < GF_ORDER; i++) er[i] = 1;
        orc_eval_poly(er, GF_ORDER);
    }
    /* scale received rows, zero the rest */
    for (size_t i = 0; i < rows; i++) {
        uint8_t *r = row_ptr(w, blocks, i);
        if (i < end && got[i]) E_mul(r, blocks, er[i]);
        else memset(r, 0, blocks * 64);
    }
    E_ifft(w, blocks, 0, rows, end, 0);
    orc_formal_derivative(w, blocks, rows);
    E_fft(w, blocks, 0, rows, end, 0);
    for (size_t i = 0; i < N; i++) {
        size_t p = orig_base + i;
        if (!got[p]) {
            E_mul(row_ptr(w, blocks, p), blocks, (gf)(GF_MOD - er[p]));
            extract_shard(w, blocks, p, restored + i * S, S);
        }
    }
    free(got); free(er);
    return E_OK;
}

/* ------------------------------------------------------------------ */
/* ChaCha8 keystream with rand_core 0.6 BlockRng fill semantics:       */
/* key = 32 x seed, 64-bit block counter from 0, stream 0; every fill  */
/* of L bytes consumes ceil(L/4) words (partial word tail discarded).   */

typedef struct { uint32_t key[8]; uint64_t block; uint32_t buf[16]; uint32_t idx; } chacha8;

static inline uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
#define QR(a, b, c, d) \
    a += b; d ^= a; d = rotl(d, 16); c += d; b ^= c; b = rotl(b, 12); \
    a += b; d ^= a; d = rotl(d, 8);  c += d; b ^= c; b = rotl(b, 7);

static void chacha8_block(chacha8 *c) {
    uint32_t in[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};
    for (int i = 0; i < 8; i++) in[4 + i] = c->key[i];
    in[12] = (uint32_t)c->block; in[13] = (uint32_t)(c->block >> 32); in[14] = 0; in[15] = 0;
    uint32_t x[16];
    memcpy(x, in, sizeof x);
    for (int r = 0; r < 4; r++) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
        QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
        QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; i++) c->buf[i] = x[i] + in[i];
    c->block++;
    c->idx = 0;
}

static void chacha8_fill(chacha8 *c, uint8_t *out, size_t len) {
    size_t done = 0;
    while (done < len) {
        if (c->idx >= 16) chacha8_block(c);
        uint32_t w = c->buf[c->idx++];
        for (int k = 0; k < 4 && done < len; k++) out[done++] = (uint8_t)(w >> (8 * k));
    }
}

/* test_util.rs:76-87 generate_original(count, shard_bytes, seed) */
void orc_generate_original(size_t count, size_t S, uint8_t seed, uint8_t *out) {
    chacha8 c;
    memset(&c, 0, sizeof c);
    uint32_t kw = seed * 0x01010101u;
    for (int i = 0; i < 8; i++) c.key[i] = kw;
    c.idx = 16;
    for (size_t i = 0; i < count; i++) chacha8_fill(&c, out + i * S, S);
}
