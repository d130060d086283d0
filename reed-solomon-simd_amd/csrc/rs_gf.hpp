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
    // low output plane: words 0-4 (from low byte), 10-14 (from high byte)
    uint32_t pl = xor3(acc_l, __builtin_amdgcn_perm(t[1], t[0], l0), __builtin_amdgcn_perm(t[3], t[2], l1));
    pl = xor3(pl, __builtin_amdgcn_perm(t[4], t[4], l2), __builtin_amdgcn_perm(t[11], t[10], h0));
    acc_l = xor3(pl, __builtin_amdgcn_perm(t[13], t[12], h1), __builtin_amdgcn_perm(t[14], t[14], h2));
    // high output plane: words 5-9, 15-19
    uint32_t ph = xor3(acc_h, __builtin_amdgcn_perm(t[6], t[5], l0), __builtin_amdgcn_perm(t[8], t[7], l1));
    ph = xor3(ph, __builtin_amdgcn_perm(t[9], t[9], l2), __builtin_amdgcn_perm(t[16], t[15], h0));
    acc_h = xor3(ph, __builtin_amdgcn_perm(t[18], t[17], h1), __builtin_amdgcn_perm(t[19], t[19], h2));
}

__device__ __forceinline__ void gf_mul4(uint32_t &xl, uint32_t &xh, const uint32_t *__restrict__ t) {
    uint32_t l = 0, h = 0;
    gf_muladd4(l, h, xl, xh, t);
    xl = l;
    xh = h;
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
