// Device-side GF(2^16) primitives shared by the MI355X kernels.
//
// Multiplication by a constant is GF(2)-linear, so x*m is the XOR of table
// lookups on 3-bit fields of x.  Four elements are packed as one 32-bit word
// of low bytes + one of high bytes (the reference's block layout,
// src/algorithm.md:18-31), and v_perm_b32 performs 4 byte lookups into an
// 8-entry table at once (12 v_perm + 8 field extracts + 6 v_bitop3 XOR3 per
// 4 elements).  A table is kPermWords = 20 words (gf_tables.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace rs {

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// The value of lane ^ 2^J of a wave64: DPP within rows of 16 lanes (J < 4),
// v_permlane16/32_swap across them (no LDS traffic).
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
    if constexpr (J == 0) return __builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    else if constexpr (J == 1) return __builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    else if constexpr (J == 2)  // lane ^ 4 = row_half_mirror (lane ^ 7) of quad_perm 3,2,1,0 (lane ^ 3):
        // two DPP moves instead of a ds_swizzle, whose lgkmcnt wait would also
        // drain LDS reads in flight
        return __builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, int(v), 0x1B, 0xF, 0xF, false), 0x141, 0xF,
                                           0xF, false);
    else return __builtin_amdgcn_update_dpp(0, int(v), 0x128, 0xF, 0xF, false);  // row_ror:8 = lane ^ 8
}
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, uint32_t lane) {
    if constexpr (J == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16u) ? r[0] : r[1];
    } else if constexpr (J == 5) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32u) ? r[0] : r[1];
    } else {
        return xor_lane<J>(v);
    }
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc_l ^= (xl,xh)*m (low plane), acc_h ^= (high plane); t = 20-word perm table
__device__ __forceinline__ void gf_muladd4(uint32_t &acc_l, uint32_t &acc_h, uint32_t xl, uint32_t xh,
                                           const uint32_t *__restrict__ t) {
    // fields 1 and 2 of both planes by one 64-bit shift each (v_lshrrev_b64):
    // the high plane's bits that enter the low word's top byte are masked off
    uint64_t x3, x6;
    const uint64_t x = (uint64_t(xh) << 32) | xl;
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(x3) : "v"(x));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(x6) : "v"(x));
    const uint32_t l0 = xl & 0x07070707u;
    const uint32_t l1 = uint32_t(x3) & 0x07070707u;
    const uint32_t l2 = uint32_t(x6) & 0x03030303u;
    const uint32_t h0 = xh & 0x07070707u;
    const uint32_t h1 = uint32_t(x3 >> 32) & 0x07070707u;
    const uint32_t h2 = uint32_t(x6 >> 32) & 0x03030303u;
    // low output plane: words 0-4 (from low byte), 10-14 (from high byte); the
    // XOR tree is two levels deep (the butterflies of a layer are latency-bound)
    const uint32_t la = xor3(__builtin_amdgcn_perm(t[1], t[0], l0), __builtin_amdgcn_perm(t[3], t[2], l1),
                             __builtin_amdgcn_perm(t[4], t[4], l2));
    const uint32_t lb = xor3(__builtin_amdgcn_perm(t[11], t[10], h0), __builtin_amdgcn_perm(t[13], t[12], h1),
                             __builtin_amdgcn_perm(t[14], t[14], h2));
    acc_l = xor3(acc_l, la, lb);
    // high output plane: words 5-9, 15-19
    const uint32_t ha = xor3(__builtin_amdgcn_perm(t[6], t[5], l0), __builtin_amdgcn_perm(t[8], t[7], l1),
                             __builtin_amdgcn_perm(t[9], t[9], l2));
    const uint32_t hb = xor3(__builtin_amdgcn_perm(t[16], t[15], h0), __builtin_amdgcn_perm(t[18], t[17], h1),
                             __builtin_amdgcn_perm(t[19], t[19], h2));
    acc_h = xor3(acc_h, ha, hb);
}

// Two pieces (fields f, f + 1) of a 16-word 2-element table from one 16-byte piece
// (A_f, C_f, A_f+1, C_f+1) of its 8-word basis (rs_codec.cpp basis_images): field
// f's four lookups are {0, a, b, a ^ b}, so A = a | b << 16 gives the table words
// [0, a_lo, b_lo, (a^b)_lo] and [0, a_hi, b_hi, (a^b)_hi] (gf_tables.cpp fill_perm2).
__device__ __forceinline__ void basis2_expand(const uint4 &v, uint4 &a, uint4 &b) {
    auto field = [](uint32_t A, uint32_t C) {
        const uint32_t tA = A ^ __builtin_amdgcn_alignbit(A, A, 16), tC = C ^ __builtin_amdgcn_alignbit(C, C, 16);
        return uint4{__builtin_amdgcn_perm(tA, A, 0x0402000Cu), __builtin_amdgcn_perm(tC, C, 0x0503010Cu),
                     __builtin_amdgcn_perm(tC, C, 0x0402000Cu), __builtin_amdgcn_perm(tA, A, 0x0503010Cu)};
    };
    a = field(v.x, v.y);
    b = field(v.z, v.w);
}

// The 20-word table of a multiplier from its 8-word basis (rs_codec.cpp
// basis_images / basis tables): multiplication by a constant is GF(2)-linear, so
// a 3-bit field's 8 lookups are [0, p0, p1, p0^p1] and that word XOR p2
// (byte O of the products pj = x * e_8B+j of input byte B).  Basis words, per
// input byte B: 4B = P0 | P1 << 16, 4B + 1 = P3 | P4 << 16, 4B + 2 = P6 | P7 << 16,
// 4B + 3 = P2 | P5 << 16.  Output: table pieces o[0..4] (words 4q .. 4q + 3 of
// fill_perm's layout, gf_tables.cpp).  ~44 VALU for 32 of the table's 80 bytes.
__device__ __forceinline__ void basis4_expand(const uint4 &b0, const uint4 &b1, uint4 (&o)[5]) {
    const uint32_t X[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    uint32_t w[20];
#pragma unroll
    for (int B = 0; B < 2; ++B) {
        const uint32_t X01 = X[4 * B], X34 = X[4 * B + 1], X67 = X[4 * B + 2], Y = X[4 * B + 3];
        const uint32_t t01 = X01 ^ __builtin_amdgcn_alignbit(X01, X01, 16);
        const uint32_t t34 = X34 ^ __builtin_amdgcn_alignbit(X34, X34, 16);
        const uint32_t t67 = X67 ^ __builtin_amdgcn_alignbit(X67, X67, 16);
#pragma unroll
        for (int O = 0; O < 2; ++O) {
            const uint32_t sel = O ? 0x0503010Cu : 0x0402000Cu;
            const uint32_t r2 = O ? 0x01010101u : 0x00000000u, r5 = O ? 0x03030303u : 0x02020202u;
            uint32_t *t = w + (2 * B + O) * 5;
            t[0] = __builtin_amdgcn_perm(t01, X01, sel);
            t[1] = t[0] ^ __builtin_amdgcn_perm(Y, Y, r2);
            t[2] = __builtin_amdgcn_perm(t34, X34, sel);
            t[3] = t[2] ^ __builtin_amdgcn_perm(Y, Y, r5);
            t[4] = __builtin_amdgcn_perm(t67, X67, sel);
        }
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) o[q] = uint4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
}

__device__ __forceinline__ void gf_mul4(uint32_t &xl, uint32_t &xh, const uint32_t *__restrict__ t) {
    uint32_t l = 0, h = 0;
    gf_muladd4(l, h, xl, xh, t);
    xl = l;
    xh = h;
}

// 2-element format (gf_tables.cpp fill_perm2): x = [lo0 lo1 hi0 hi1], t = 16
// words.  Per 2-bit field f: a "direct" lookup on the field values in place
// (low-byte fields -> low output bytes, high-byte fields -> high output bytes)
// and a "cross" lookup on the word rotated by 16 bits (high-byte fields -> low
// output bytes and vice versa); selectors of the high half index the table's
// upper 4 bytes (+4).  12 field ops, 8 v_perm, 4 v_bitop3 XOR3 per 2 elements.
__device__ __forceinline__ void gf_muladd2(uint32_t &acc, uint32_t x, const uint32_t *__restrict__ t) {
    const uint32_t xr = __builtin_amdgcn_alignbit(x, x, 16);
    const uint64_t xx = (uint64_t(xr) << 32) | x;
    uint64_t x2, x4, x6;
    asm("v_lshrrev_b64 %0, 2, %1" : "=v"(x2) : "v"(xx));
    asm("v_lshrrev_b64 %0, 4, %1" : "=v"(x4) : "v"(xx));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(x6) : "v"(xx));
    // (v & M) | C in one v_bitop3 (truth table 0xEA = S0 & S1 | S2): VOP3 takes no
    // literal, so the compiler keeps M and C in registers
    constexpr uint32_t M = 0x03030303u, C = 0x04040000u;
    auto sel = [](uint32_t v) { return __builtin_amdgcn_bitop3_b32(v, M, C, 0xEA); };
    const uint32_t d0 = sel(x), c0 = sel(xr);
    const uint32_t d1 = sel(uint32_t(x2)), c1 = sel(uint32_t(x2 >> 32));
    const uint32_t d2 = sel(uint32_t(x4)), c2 = sel(uint32_t(x4 >> 32));
    const uint32_t d3 = sel(uint32_t(x6)), c3 = sel(uint32_t(x6 >> 32));
    const uint32_t a = xor3(__builtin_amdgcn_perm(t[1], t[0], d0), __builtin_amdgcn_perm(t[3], t[2], c0),
                            __builtin_amdgcn_perm(t[5], t[4], d1));
    const uint32_t b = xor3(__builtin_amdgcn_perm(t[7], t[6], c1), __builtin_amdgcn_perm(t[9], t[8], d2),
                            __builtin_amdgcn_perm(t[11], t[10], c2));
    const uint32_t c = xor3(acc, __builtin_amdgcn_perm(t[13], t[12], d3), __builtin_amdgcn_perm(t[15], t[14], c3));
    acc = xor3(a, b, c);
}

__device__ __forceinline__ void gf_mul2(uint32_t &x, const uint32_t *__restrict__ t) {
    uint32_t acc = 0;
    gf_muladd2(acc, x, t);
    x = acc;
}

__device__ __forceinline__ void ifft_bfly2(uint32_t &a, uint32_t &b, const uint32_t *__restrict__ t) {
    b ^= a;
    gf_muladd2(a, b, t);
}

__device__ __forceinline__ void fft_bfly2(uint32_t &a, uint32_t &b, const uint32_t *__restrict__ t) {
    gf_muladd2(a, b, t);
    b ^= a;
}

// IFFT butterfly (engine_naive.rs:96-100): b ^= a; a ^= b * m
__device__ __forceinline__ void ifft_bfly(uint32_t &al, uint32_t &ah, uint32_t &bl, uint32_t &bh,
                                          const uint32_t *__restrict__ t) {
    bl ^= al;
    bh ^= ah;
    gf_muladd4(al, ah, bl, bh, t);
}

// FFT butterfly (engine_naive.rs:64-68): a ^= b * m; b ^= a
__device__ __forceinline__ void fft_bfly(uint32_t &al, uint32_t &ah, uint32_t &bl, uint32_t &bh,
                                         const uint32_t *__restrict__ t) {
    gf_muladd4(al, ah, bl, bh, t);
    bl ^= al;
    bh ^= ah;
}

}  // namespace rs
