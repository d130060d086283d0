// GF(2^16) table construction (host).  Semantics follow reference
// src/engine/tables.rs (exp/log :184-221, log_walsh :223-233, skew :285-324,
// mul :172-178); the byte-permute tables are this engine's own format.
#include "gf_tables.hpp"
#include "rs_device.hpp"

#include <mutex>

namespace rs {

namespace {

constexpr uint16_t kCantorBasis[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                       0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
constexpr uint32_t kPoly = 0x1002D;

// In-place Walsh-Hadamard transform of 2^u values over Z/65535.
void walsh(uint16_t *v, uint32_t n) {
    for (uint32_t half = 1; half < n; half *= 2)
        for (uint32_t blk = 0; blk < n; blk += 2 * half)
            for (uint32_t k = blk; k < blk + half; ++k) {
                const uint16_t p = v[k], q = v[k + half];
                v[k] = add_mod(p, q);
                v[k + half] = sub_mod(p, q);
            }
}

// Fill one byte-permute table for the linear map x -> f(x).
//
// Layout (PermTable, kPermWords = 20 words): for input byte plane B (0 = low
// byte of the element, 1 = high byte) and output plane O (0 = low, 1 = high),
// the 5 words at [(2B + O) * 5] are
//   w0,w1 : bits 0-2 of the input byte  -> 8 output bytes (v_perm selector 0..7)
//   w2,w3 : bits 3-5                     -> 8 output bytes
//   w4    : bits 6-7                     -> 4 output bytes (selector 0..3)
// so that a v_perm_b32 on 4 packed selector bytes looks up 4 elements at once.
template <typename F>
void fill_perm(uint32_t *w, F f) {
    for (int B = 0; B < 2; ++B)
        for (int O = 0; O < 2; ++O) {
            uint32_t *t = w + (2 * B + O) * 5;
            const int shifts[3] = {0, 3, 6};
            const int entries[3] = {8, 8, 4};
            int word = 0;
            for (int g = 0; g < 3; ++g) {
                uint8_t bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                for (int k = 0; k < entries[g]; ++k) {
                    const uint16_t x = static_cast<uint16_t>(k << (8 * B + shifts[g]));
                    const uint16_t p = f(x);
                    bytes[k] = static_cast<uint8_t>(O ? (p >> 8) : (p & 0xFF));
                }
                for (int q = 0; q < entries[g] / 4; ++q)
                    t[word++] = bytes[4 * q] | (bytes[4 * q + 1] << 8) | (bytes[4 * q + 2] << 16) |
                                (static_cast<uint32_t>(bytes[4 * q + 3]) << 24);
            }
        }
}

// 2-element format (kPerm2Words = 16 words): a word holds the low bytes of 2
// elements in bytes 0-1 and their high bytes in bytes 2-3.  For each 2-bit
// field f (bits 2f, 2f+1) of an input byte, two v_perm_b32 tables of 8 bytes:
//   words [4f, 4f+1]   "direct": bytes 0-3 = low output byte of the LOW-byte
//                       field's 4 values, bytes 4-7 = high output byte of the
//                       HIGH-byte field's (selector [lo0 lo1 hi0+4 hi1+4])
//   words [4f+2, 4f+3] "cross":  bytes 0-3 = low output byte of the HIGH-byte
//                       field, bytes 4-7 = high output byte of the LOW-byte
//                       field (selector of the word rotated by 16 bits)
// (v_perm_b32 S0, S1: selector bytes 0-3 pick S1's bytes, 4-7 S0's, so the
// first word of each pair is S1).
template <typename F>
void fill_perm2(uint32_t *w, F f) {
    for (int fld = 0; fld < 4; ++fld) {
        uint8_t direct[8], cross[8];
        for (int v = 0; v < 4; ++v) {
            const uint16_t plo = f(static_cast<uint16_t>(v << (2 * fld)));      // low-byte field
            const uint16_t phi = f(static_cast<uint16_t>(v << (8 + 2 * fld)));  // high-byte field
            direct[v] = static_cast<uint8_t>(plo & 0xFF);
            direct[4 + v] = static_cast<uint8_t>(phi >> 8);
            cross[v] = static_cast<uint8_t>(phi & 0xFF);
            cross[4 + v] = static_cast<uint8_t>(plo >> 8);
        }
        auto word = [](const uint8_t *b) {
            return b[0] | (b[1] << 8) | (b[2] << 16) | (static_cast<uint32_t>(b[3]) << 24);
        };
        w[4 * fld + 0] = word(direct);
        w[4 * fld + 1] = word(direct + 4);
        w[4 * fld + 2] = word(cross);
        w[4 * fld + 3] = word(cross + 4);
    }
}

GfTables *build() {
    auto *T = new GfTables;
    T->exp.assign(kOrder, 0);
    T->log.assign(kOrder, 0);

    // discrete log in polynomial basis from the LFSR sequence
    std::vector<uint16_t> lfsr_log(kOrder);
    uint32_t state = 1;
    for (uint32_t e = 0; e < kModulus; ++e) {
        lfsr_log[state] = static_cast<uint16_t>(e);
        state <<= 1;
        if (state & kOrder) state ^= kPoly;
    }
    lfsr_log[0] = kModulus;
    // Cantor coordinate c -> polynomial element -> log
    std::vector<uint16_t> elem(kOrder, 0);
    for (int bit = 0; bit < 16; ++bit)
        for (uint32_t c = 0; c < (1u << bit); ++c) elem[c | (1u << bit)] = elem[c] ^ kCantorBasis[bit];
    for (uint32_t c = 0; c < kOrder; ++c) T->log[c] = lfsr_log[elem[c]];
    for (uint32_t c = 0; c < kOrder; ++c) T->exp[T->log[c]] = static_cast<uint16_t>(c);
    T->exp[kModulus] = T->exp[0];

    // skew factors (tables.rs:285-324): additive-FFT twiddles, stored as logs
    std::vector<uint16_t> raw(kModulus, 0);
    uint16_t sub[15];
    for (int k = 0; k < 15; ++k) sub[k] = static_cast<uint16_t>(2u << k);
    for (int m = 0; m < 15; ++m) {
        raw[(1u << m) - 1] = 0;
        for (int i = m; i < 15; ++i) {
            const uint32_t span = 2u << i;
            for (uint32_t j = (1u << m) - 1; j < span; j += 2u << m) raw[j + span] = raw[j] ^ sub[i];
        }
        sub[m] = static_cast<uint16_t>(kModulus - T->log[T->mul(sub[m], T->log[sub[m] ^ 1])]);
        for (int i = m + 1; i < 15; ++i) sub[i] = T->mul(sub[i], add_mod(T->log[sub[i] ^ 1], sub[m]));
    }
    T->skew.assign(kOrder, kModulus);
    for (uint32_t i = 0; i < kModulus; ++i) T->skew[i] = T->log[raw[i]];

    // log_walsh: Walsh transform of log[] with log[0] := 0
    T->log_walsh = T->log;
    T->log_walsh[0] = 0;
    walsh(T->log_walsh.data(), kOrder);

    // folded log_walsh for the reduced eval_poly (see DESIGN.md "eval_poly")
    T->lw_fold.assign(2 * kOrder - 1, 0);
    for (int u = 0; u <= 16; ++u) {
        const uint32_t n = 1u << u;
        uint16_t *dst = &T->lw_fold[n - 1];
        for (uint32_t i = 0; i < kOrder; ++i) dst[i & (n - 1)] = add_mod(dst[i & (n - 1)], T->log_walsh[i]);
    }

    // byte-permute multiply tables
    T->perm_by_log.assign(size_t(kOrder) * kPermWords, 0);
    T->perm_by_skew.assign(size_t(kOrder) * kPermWords, 0);
    for (uint32_t lm = 0; lm < kOrder; ++lm)
        fill_perm(&T->perm_by_log[size_t(lm) * kPermWords],
                  [&](uint16_t x) { return T->mul(x, static_cast<uint16_t>(lm)); });
    for (uint32_t idx = 0; idx < kOrder; ++idx) {
        const uint16_t lm = T->skew[idx];
        if (lm == kModulus) continue;  // multiply-by-zero: all-zero table
        std::copy_n(&T->perm_by_log[size_t(lm) * kPermWords], kPermWords, &T->perm_by_skew[size_t(idx) * kPermWords]);
    }
    T->perm2_by_log.assign(size_t(kOrder) * kPerm2Words, 0);
    T->perm2_by_skew.assign(size_t(kOrder) * kPerm2Words, 0);
    for (uint32_t lm = 0; lm < kOrder; ++lm)
        fill_perm2(&T->perm2_by_log[size_t(lm) * kPerm2Words],
                   [&](uint16_t x) { return T->mul(x, static_cast<uint16_t>(lm)); });
    for (uint32_t idx = 0; idx < kOrder; ++idx) {
        const uint16_t lm = T->skew[idx];
        if (lm == kModulus) continue;
        std::copy_n(&T->perm2_by_log[size_t(lm) * kPerm2Words], kPerm2Words,
                    &T->perm2_by_skew[size_t(idx) * kPerm2Words]);
    }
    return T;
}

}  // namespace

// rs_device.hpp: name of the last kernel launched by this thread (profiler records)
char *launch_name_buf() {
    static thread_local char name[kLaunchNameBytes];
    return name;
}

uint16_t add_mod(uint16_t a, uint16_t b) {
    const uint32_t s = uint32_t(a) + b;
    return static_cast<uint16_t>(s + (s >> 16));
}

uint16_t sub_mod(uint16_t a, uint16_t b) {
    const uint32_t d = uint32_t(a) - uint32_t(b);
    return static_cast<uint16_t>(d + (d >> 16));
}

uint16_t GfTables::mul(uint16_t x, uint16_t log_m) const {
    return x == 0 ? 0 : exp[add_mod(log[x], log_m)];
}

const GfTables &tables() {
    static std::once_flag once;
    static GfTables *T = nullptr;
    std::call_once(once, [] { T = build(); });
    return *T;
}

void eval_poly_host(uint16_t *er, size_t /*truncated: zero past it, so the full transform is identical*/) {
    const GfTables &T = tables();
    walsh(er, kOrder);
    for (uint32_t i = 0; i < kOrder; ++i) {
        const uint32_t p = uint32_t(er[i]) * T.log_walsh[i];
        er[i] = add_mod(static_cast<uint16_t>(p), static_cast<uint16_t>(p >> 16));
    }
    walsh(er, kOrder);
}

}  // namespace rs
