/*
 * avx2_port.c -- CPU baseline: a C restatement of the reference's AVX2 engine
 * algorithm (TEST / BASELINE INFRASTRUCTURE ONLY; never linked into the product).
 *
 * Algorithm followed (paths relative to /root/reference):
 *   Mul128 nibble tables .......... src/engine/tables.rs:253-282
 *   mul_256 (4 x vpshufb / plane) . src/engine/engine_avx2.rs:162-187
 *   fftb_256 / ifftb_256 .......... src/engine/engine_avx2.rs:214-236, 358-380
 *   radix-4 "two layers at a time"  src/engine/engine_avx2.rs:250-349 (fft), 393-491 (ifft)
 *   odd final layer ............... src/engine/engine_nosimd.rs:194-211, 295-311
 * Single-threaded, like the reference.  Checked byte-identical to the radix-2
 * oracle (rs_oracle.c) and thereby to the reference's golden hashes.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

const uint16_t *orc_exp_table(void);
const uint16_t *orc_log_table(void);
const uint16_t *orc_skew_table(void);
uint16_t orc_gf_mul(uint16_t x, uint16_t log_m);

#define GF_MOD 65535u

/* per log_m: 4 nibble positions x {lo-byte, hi-byte} x 16 entries */
typedef struct { uint8_t lo[4][16]; uint8_t hi[4][16]; } nib_lut;
static nib_lut *g_lut = NULL;
static const uint16_t *g_skew = NULL;

int avx2_available(void) { return __builtin_cpu_supports("avx2"); }

static void build_luts(void) {
    if (g_lut) return;
    const uint16_t *ex = orc_exp_table(), *lg = orc_log_table();
    nib_lut *t = aligned_alloc(64, sizeof(nib_lut) * 65536);
    for (uint32_t m = 0; m < 65536; m++)
        for (int pos = 0; pos < 4; pos++)
            for (uint32_t x = 0; x < 16; x++) {
                uint16_t v = (uint16_t)(x << (4 * pos));
                uint16_t p = 0;
                if (v) {
                    uint32_t s = (uint32_t)lg[v] + m;
                    p = ex[(uint16_t)(s + (s >> 16))];
                }
                t[m].lo[pos][x] = (uint8_t)p;
                t[m].hi[pos][x] = (uint8_t)(p >> 8);
            }
    g_skew = orc_skew_table();
    g_lut = t;
}

typedef struct { __m256i l[4], h[4]; } lut256;

__attribute__((target("avx2"))) static inline lut256 load_lut(uint16_t log_m) {
    lut256 r;
    const nib_lut *t = &g_lut[log_m];
    for (int i = 0; i < 4; i++) {
        r.l[i] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t->lo[i]));
        r.h[i] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t->hi[i]));
    }
    return r;
}

/* product of the 32 elements (lo plane, hi plane) by the table's constant */
__attribute__((target("avx2"))) static inline void mul256(__m256i vlo, __m256i vhi, const lut256 *t,
                                                          __m256i *plo, __m256i *phi) {
    const __m256i nib = _mm256_set1_epi8(0x0f);
    __m256i n0 = _mm256_and_si256(vlo, nib);
    __m256i n1 = _mm256_and_si256(_mm256_srli_epi64(vlo, 4), nib);
    __m256i n2 = _mm256_and_si256(vhi, nib);
    __m256i n3 = _mm256_and_si256(_mm256_srli_epi64(vhi, 4), nib);
    __m256i lo = _mm256_shuffle_epi8(t->l[0], n0);
    __m256i hi = _mm256_shuffle_epi8(t->h[0], n0);
    lo = _mm256_xor_si256(lo, _mm256_shuffle_epi8(t->l[1], n1));
    hi = _mm256_xor_si256(hi, _mm256_shuffle_epi8(t->h[1], n1));
    lo = _mm256_xor_si256(lo, _mm256_shuffle_epi8(t->l[2], n2));
    hi = _mm256_xor_si256(hi, _mm256_shuffle_epi8(t->h[2], n2));
    lo = _mm256_xor_si256(lo, _mm256_shuffle_epi8(t->l[3], n3));
    hi = _mm256_xor_si256(hi, _mm256_shuffle_epi8(t->h[3], n3));
    *plo = lo;
    *phi = hi;
}

#define ROW(d, blocks, r) ((d) + (size_t)(r) * (blocks) * 64)

__attribute__((target("avx2"))) static void xor_rows(uint8_t *x, const uint8_t *y, size_t blocks) {
    for (size_t b = 0; b < blocks * 2; b++) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(x + 32 * b));
        __m256i c = _mm256_loadu_si256((const __m256i *)(y + 32 * b));
        _mm256_storeu_si256((__m256i *)(x + 32 * b), _mm256_xor_si256(a, c));
    }
}

/* FFT butterfly on two rows: x ^= y*m ; y ^= x   (65535 => XOR only) */
__attribute__((target("avx2"))) static void fft_bfly(uint8_t *x, uint8_t *y, size_t blocks, uint16_t lm) {
    if (lm == GF_MOD) { xor_rows(y, x, blocks); return; }
    lut256 t = load_lut(lm);
    for (size_t b = 0; b < blocks; b++) {
        __m256i *px = (__m256i *)(x + 64 * b), *py = (__m256i *)(y + 64 * b);
        __m256i xl = _mm256_loadu_si256(px), xh = _mm256_loadu_si256(px + 1);
        __m256i yl = _mm256_loadu_si256(py), yh = _mm256_loadu_si256(py + 1);
        __m256i pl, ph;
        mul256(yl, yh, &t, &pl, &ph);
        xl = _mm256_xor_si256(xl, pl);
        xh = _mm256_xor_si256(xh, ph);
        _mm256_storeu_si256(px, xl);
        _mm256_storeu_si256(px + 1, xh);
        _mm256_storeu_si256(py, _mm256_xor_si256(yl, xl));
        _mm256_storeu_si256(py + 1, _mm256_xor_si256(yh, xh));
    }
}

/* IFFT butterfly on two rows: y ^= x ; x ^= y*m */
__attribute__((target("avx2"))) static void ifft_bfly(uint8_t *x, uint8_t *y, size_t blocks, uint16_t lm) {
    if (lm == GF_MOD) { xor_rows(y, x, blocks); return; }
    lut256 t = load_lut(lm);
    for (size_t b = 0; b < blocks; b++) {
        __m256i *px = (__m256i *)(x + 64 * b), *py = (__m256i *)(y + 64 * b);
        __m256i xl = _mm256_loadu_si256(px), xh = _mm256_loadu_si256(px + 1);
        __m256i yl = _mm256_xor_si256(_mm256_loadu_si256(py), xl);
        __m256i yh = _mm256_xor_si256(_mm256_loadu_si256(py + 1), xh);
        __m256i pl, ph;
        mul256(yl, yh, &t, &pl, &ph);
        _mm256_storeu_si256(py, yl);
        _mm256_storeu_si256(py + 1, yh);
        _mm256_storeu_si256(px, _mm256_xor_si256(xl, pl));
        _mm256_storeu_si256(px + 1, _mm256_xor_si256(xh, ph));
    }
}

void avx2_fft(uint8_t *d, size_t blocks, size_t pos, size_t size, size_t trunc, size_t delta) {
    build_luts();
    size_t dist4 = size, dist = size >> 2;
    for (; dist != 0; dist4 = dist, dist >>= 2)
        for (size_t r = 0; r < trunc; r += dist4) {
            size_t base = r + dist + delta - 1;
            uint16_t m01 = g_skew[base], m02 = g_skew[base + dist], m23 = g_skew[base + 2 * dist];
            for (size_t i = r; i < r + dist; i++) {
                uint8_t *s0 = ROW(d, blocks, pos + i), *s1 = ROW(d, blocks, pos + i + dist);
                uint8_t *s2 = ROW(d, blocks, pos + i + 2 * dist), *s3 = ROW(d, blocks, pos + i + 3 * dist);
                fft_bfly(s0, s2, blocks, m02);
                fft_bfly(s1, s3, blocks, m02);
                fft_bfly(s0, s1, blocks, m01);
                fft_bfly(s2, s3, blocks, m23);
            }
        }
    if (dist4 == 2)
        for (size_t r = 0; r < trunc; r += 2)
            fft_bfly(ROW(d, blocks, pos + r), ROW(d, blocks, pos + r + 1), blocks, g_skew[r + delta]);
}

void avx2_ifft(uint8_t *d, size_t blocks, size_t pos, size_t size, size_t trunc, size_t delta) {
    build_luts();
    size_t dist = 1, dist4 = 4;
    for (; dist4 <= size; dist = dist4, dist4 <<= 2)
        for (size_t r = 0; r < trunc; r += dist4) {
            size_t base = r + dist + delta - 1;
            uint16_t m01 = g_skew[base], m02 = g_skew[base + dist], m23 = g_skew[base + 2 * dist];
            for (size_t i = r; i < r + dist; i++) {
                uint8_t *s0 = ROW(d, blocks, pos + i), *s1 = ROW(d, blocks, pos + i + dist);
                uint8_t *s2 = ROW(d, blocks, pos + i + 2 * dist), *s3 = ROW(d, blocks, pos + i + 3 * dist);
                ifft_bfly(s0, s1, blocks, m01);
                ifft_bfly(s2, s3, blocks, m23);
                ifft_bfly(s0, s2, blocks, m02);
                ifft_bfly(s1, s3, blocks, m02);
            }
        }
    if (dist < size) {
        uint16_t lm = g_skew[dist + delta - 1];
        for (size_t i = 0; i < dist; i++) ifft_bfly(ROW(d, blocks, pos + i), ROW(d, blocks, pos + i + dist), blocks, lm);
    }
}

__attribute__((target("avx2"))) void avx2_mul(uint8_t *rows, size_t blocks, uint16_t log_m) {
    build_luts();
    lut256 t = load_lut(log_m);
    for (size_t b = 0; b < blocks; b++) {
        __m256i *p = (__m256i *)(rows + 64 * b);
        __m256i pl, ph;
        mul256(_mm256_loadu_si256(p), _mm256_loadu_si256(p + 1), &t, &pl, &ph);
        _mm256_storeu_si256(p, pl);
        _mm256_storeu_si256(p + 1, ph);
    }
}
