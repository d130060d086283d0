// HIP kernels of the MI355X (gfx950) Reed-Solomon GF(2^16) engine.
//
// The hot path is the additive FFT / IFFT of the Leopard construction over the
// shard matrix (reference: src/engine/engine_naive.rs:43-105 semantics,
// src/rate/rate_high.rs / rate_low.rs call sites).  Every engine op acts
// independently on each element column, so a transform over n rows is split
// into passes over row SETS x 64-pack column SLICES.
//
// GF multiply: multiplication by a constant is GF(2)-linear, so x*m is the XOR
// of table lookups on 3-bit fields of x.  Four elements are packed as one
// 32-bit word of low bytes + one of high bytes (the reference's block layout),
// and v_perm_b32 performs 4 byte lookups into an 8-entry table at once
// (12 v_perm + 10 field extracts + 6 v_bitop3 XOR3 per 4 elements).
// The twiddle of a butterfly group is wave-uniform: lanes run along the
// columns of one row pair, so each table arrives through scalar loads.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rs_device.hpp"

namespace rs {
namespace {

constexpr int kLanes = 64;

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
    const uint32_t l0 = xl & 0x07070707u;
    const uint32_t l1 = (xl >> 3) & 0x07070707u;
    const uint32_t l2 = (xl >> 6) & 0x03030303u;
    const uint32_t h0 = xh & 0x07070707u;
    const uint32_t h1 = (xh >> 3) & 0x07070707u;
    const uint32_t h2 = (xh >> 6) & 0x03030303u;
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

// -------------------------------------------------------------------------
// Pass kernel.  K: log2 rows per set; LR: log2 rows held per lane.
// Waves W = 2^(K-LR).  Phase A: a wave holds local rows (w << LR) | i
// (bits [0,LR) in registers).  Phase B: rows (i << (K-LR)) | w (bits
// [K-LR, K) in registers).  K <= 2*LR, so IFFT = A-layers then B-layers and
// FFT = B-layers then A-layers, with one LDS exchange each.
template <int K, int LR>
struct Pass {
    static constexpr int R = 1 << LR;
    static constexpr int W = 1 << (K - LR);
    static constexpr int kThreads = kLanes * W;
    static_assert(K <= 2 * LR, "two register phases must cover all local bits");

    template <bool PB>
    static __device__ __forceinline__ uint32_t lrow(uint32_t w, int i) {
        if constexpr (W == 1) return i;
        if constexpr (PB) return (uint32_t(i) << (K - LR)) | w;
        return (w << LR) | uint32_t(i);
    }
};

struct Ctx {
    uint32_t lane, w, s_lo, s_hi, a, pk_off;
    bool pk_ok;
    __device__ __forceinline__ uint32_t grow(uint32_t j, int K) const { return s_lo + (j << a) + (s_hi << (a + K)); }
};

template <int K, int LR, bool PB>
__device__ __forceinline__ void load_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, uint32_t (&lo)[1 << LR],
                                          uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t r = c.grow(P::template lrow<PB>(c.w, i), K) + chunk * A.n;
        const uint8_t *p = nullptr;
        if (A.work_in) {
            p = A.work_in + uint64_t(r) * A.work_stride;
        } else {
            for (uint32_t k = 0; k < A.nsrc; ++k)
                if (r >= A.src[k].row_begin && r < A.src[k].row_end)
                    p = A.src[k].base + uint64_t(r - A.src[k].row_begin) * A.src[k].stride;
        }
        uint32_t ri = 0;
        if (A.load_scale) {
            ri = A.rowinfo[r];
            if (ri & 0x10000u) p = nullptr;
        }
        uint32_t l = 0, h = 0;
        if (p && c.pk_ok) {
            l = *reinterpret_cast<const uint32_t *>(p + c.pk_off);
            h = *reinterpret_cast<const uint32_t *>(p + c.pk_off + 32);
        }
        if (A.load_scale && p) gf_mul4(l, h, A.lut + (ri & 0xFFFFu) * 20u);
        lo[i] = l;
        hi[i] = h;
    });
}

template <int K, int LR, bool PB>
__device__ __forceinline__ void store_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, uint32_t (&lo)[1 << LR],
                                           uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t r = c.grow(P::template lrow<PB>(c.w, i), K) + chunk * A.n;
        uint8_t *p = nullptr;
        uint32_t l = lo[i], h = hi[i];
        if (A.work_out) {
            p = A.work_out + uint64_t(r) * A.work_stride;
        } else if (r >= A.dst.row_begin && r < A.dst.row_end) {
            p = const_cast<uint8_t *>(A.dst.base) + uint64_t(r - A.dst.row_begin) * A.dst.stride;
            if (A.reveal) {
                const uint32_t ri = A.rowinfo[r];
                if (ri & 0x10000u) gf_mul4(l, h, A.lut + (65535u - (ri & 0xFFFFu)) * 20u);
                else p = nullptr;
            }
        }
        if (p && c.pk_ok) {
            *reinterpret_cast<uint32_t *>(p + c.pk_off) = l;
            *reinterpret_cast<uint32_t *>(p + c.pk_off + 32) = h;
        }
    });
}

// One butterfly layer on local bit B (global bit a + B), rows held in phase PB.
template <int K, int LR, bool PB, int B, bool IFFT>
__device__ __forceinline__ void layer(const PassArgs &A, const Ctx &c, uint32_t delta, uint32_t (&lo)[1 << LR],
                                      uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    constexpr int RB = PB && P::W > 1 ? B - (K - LR) : B;  // register bit
    static_assert(RB >= 0 && RB < LR, "bit not resident in this phase");
    const uint32_t gbit = c.a + B;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr ((i & (1 << RB)) == 0) {
            constexpr int i2 = i | (1 << RB);
            const uint32_t g = c.grow(P::template lrow<PB>(c.w, i), K);
            const uint32_t r = g & ~((2u << gbit) - 1u);
            const uint32_t idx = r + (1u << gbit) + delta - 1u;
            const uint32_t *t = A.tw + idx * 20u;
            if constexpr (IFFT) ifft_bfly(lo[i], hi[i], lo[i2], hi[i2], t);
            else fft_bfly(lo[i], hi[i], lo[i2], hi[i2], t);
        }
    });
}

template <int K, int LR, bool FROM_B, bool TO_B>
__device__ __forceinline__ void exchange(const Ctx &c, uint32_t *lds, uint32_t (&lo)[1 << LR],
                                         uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    if constexpr (P::W == 1 || FROM_B == TO_B) return;
    uint32_t *llo = lds, *lhi = lds + (kLanes << K);
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<FROM_B>(c.w, i);
        llo[j * kLanes + c.lane] = lo[i];
        lhi[j * kLanes + c.lane] = hi[i];
    });
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<TO_B>(c.w, i);
        lo[i] = llo[j * kLanes + c.lane];
        hi[i] = lhi[j * kLanes + c.lane];
    });
}

// Formal derivative restricted to the set's local bits:
//   x[q] <- (mode 2 ? x[q] : 0) ^ XOR_{b < K, q_b = 0} x[q | 2^b]
template <int K, int LR, bool PB>
__device__ __forceinline__ void formal_derivative(const Ctx &c, uint32_t mode, uint32_t *lds,
                                                  uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    uint32_t *llo = lds, *lhi = lds + (kLanes << K);
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<PB>(c.w, i);
        llo[j * kLanes + c.lane] = lo[i];
        lhi[j * kLanes + c.lane] = hi[i];
    });
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<PB>(c.w, i);
        uint32_t l = mode == 2 ? lo[i] : 0u, h = mode == 2 ? hi[i] : 0u;
#pragma unroll
        for (int b = 0; b < K; ++b)
            if (!(j & (1u << b))) {
                l ^= llo[(j | (1u << b)) * kLanes + c.lane];
                h ^= lhi[(j | (1u << b)) * kLanes + c.lane];
            }
        lo[i] = l;
        hi[i] = h;
    });
}

template <int K, int LR, bool PB>
__device__ __forceinline__ void xor_rows_in(const PassArgs &A, const Ctx &c, uint32_t (&lo)[1 << LR],
                                            uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t r = c.grow(P::template lrow<PB>(c.w, i), K);
        const uint8_t *p = A.xor_in + uint64_t(r) * A.work_stride;
        if (c.pk_ok) {
            lo[i] ^= *reinterpret_cast<const uint32_t *>(p + c.pk_off);
            hi[i] ^= *reinterpret_cast<const uint32_t *>(p + c.pk_off + 32);
        }
    });
}

template <int K, int LR, int FLAGS>
__global__ void __launch_bounds__(kLanes << (K - LR)) k_pass(const PassArgs A) {
    using P = Pass<K, LR>;
    constexpr bool DO_IFFT = FLAGS & kIfft;
    constexpr bool DO_FFT = FLAGS & kFft;
    constexpr bool HAS_B = P::W > 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    Ctx c;
    c.lane = threadIdx.x & (kLanes - 1);
    c.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t slice = blockIdx.x % A.slices;
    const uint32_t set = blockIdx.x / A.slices;
    const uint32_t gchunk = blockIdx.y;
    c.a = A.a;
    c.s_lo = set & ((1u << A.a) - 1u);
    c.s_hi = set >> A.a;
    const uint32_t pk = slice * kLanes + c.lane;
    c.pk_ok = pk < A.packs;
    c.pk_off = (pk >> 3) * 64u + (pk & 7u) * 4u;

    uint32_t lo[P::R], hi[P::R];

    // ---- load (+ IFFT per input chunk, XOR-accumulated) ------------------
    if constexpr (DO_IFFT) {
        uint32_t tl[P::R], th[P::R];
        for (uint32_t ci = 0; ci < A.in_chunks; ++ci) {
            const uint32_t chunk = gchunk + ci;
            load_rows<K, LR, false>(A, c, chunk, tl, th);
            const uint32_t delta = A.ifft_delta + chunk * A.ifft_delta_step;
            static_for<0, LR < K ? LR : K>([&](auto bc) { layer<K, LR, false, decltype(bc)::value, true>(A, c, delta, tl, th); });
            if constexpr (HAS_B) {
                exchange<K, LR, false, true>(c, lds, tl, th);
                static_for<LR, K>([&](auto bc) { layer<K, LR, true, decltype(bc)::value, true>(A, c, delta, tl, th); });
            }
            if (ci == 0) {
                static_for<0, P::R>([&](auto ic) { lo[ic] = tl[ic]; hi[ic] = th[ic]; });
            } else {
                static_for<0, P::R>([&](auto ic) { lo[ic] ^= tl[ic]; hi[ic] ^= th[ic]; });
            }
        }
    } else {
        load_rows<K, LR, HAS_B>(A, c, gchunk, lo, hi);
    }
    // rows are now in phase B (if the pass has one)

    if (A.fd_mode) formal_derivative<K, LR, HAS_B>(c, A.fd_mode, lds, lo, hi);
    if (A.xor_in) xor_rows_in<K, LR, HAS_B>(A, c, lo, hi);

    // ---- FFT per output chunk + store ------------------------------------
    if constexpr (DO_FFT) {
        for (uint32_t co = 0; co < A.out_chunks; ++co) {
            const uint32_t chunk = gchunk + co;
            const uint32_t delta = A.fft_delta + chunk * A.fft_delta_step;
            uint32_t yl[P::R], yh[P::R];
            static_for<0, P::R>([&](auto ic) { yl[ic] = lo[ic]; yh[ic] = hi[ic]; });
            if constexpr (HAS_B) {
                static_for<0, K - LR>([&](auto bc) {
                    constexpr int b = K - 1 - decltype(bc)::value;
                    layer<K, LR, true, b, false>(A, c, delta, yl, yh);
                });
                exchange<K, LR, true, false>(c, lds, yl, yh);
                static_for<0, LR>([&](auto bc) {
                    constexpr int b = LR - 1 - decltype(bc)::value;
                    layer<K, LR, false, b, false>(A, c, delta, yl, yh);
                });
            } else {
                static_for<0, K>([&](auto bc) {
                    constexpr int b = K - 1 - decltype(bc)::value;
                    layer<K, LR, false, b, false>(A, c, delta, yl, yh);
                });
            }
            store_rows<K, LR, false>(A, c, chunk, yl, yh);
        }
    } else {
        store_rows<K, LR, HAS_B>(A, c, gchunk, lo, hi);
    }
}

// Note on phases: with HAS_B the IFFT leaves rows in phase B and the FFT ends
// in phase A; without FFT the store happens in phase B.  The layer bits in
// phase B are [K-LR, K): the IFFT's B-layers run over [LR, K) which is inside
// it because K <= 2*LR.  The FFT's B-layers run over [LR, K) as well
// (descending), its A-layers over [0, LR).

template <int K, int LR, int F>
hipError_t launch_f(const PassArgs &A, hipStream_t s) {
    using P = Pass<K, LR>;
    // LDS: one [2^K rows][64 lanes] tile of low words + one of high words
    const size_t lds = size_t(8) * kLanes << K;
    static bool attr_set = false;  // benign race: idempotent attribute call
    if (!attr_set && lds > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pass<K, LR, F>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    dim3 grid(A.slices * A.nsets, A.grid_chunks);
    k_pass<K, LR, F><<<grid, P::kThreads, lds, s>>>(A);
    return hipGetLastError();
}

template <int K, int LR>
hipError_t launch_k(int flags, const PassArgs &A, hipStream_t s) {
    switch (flags) {
        case kIfft: return launch_f<K, LR, kIfft>(A, s);
        case kFft: return launch_f<K, LR, kFft>(A, s);
        case kIfft | kFft: return launch_f<K, LR, kIfft | kFft>(A, s);
        default: return launch_f<K, LR, 0>(A, s);
    }
}

// ---------------------------------------------------------------------------
// eval_poly (reference src/engine/utils.rs:20-31) reduced to 2^u points:
// the erasure vector is zero outside [0, 2^u) (high rate) or equals 1 there
// (low rate), so FWHT_16 collapses onto 2^u residues (DESIGN.md "eval_poly").
__device__ __forceinline__ uint32_t add_mod(uint32_t a, uint32_t b) {
    const uint32_t s = a + b;
    return (s + (s >> 16)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t sub_mod(uint32_t a, uint32_t b) {
    const uint32_t d = a - b;
    return (d + (d >> 16)) & 0xFFFFu;
}

__device__ void walsh_lds(uint16_t *v, uint32_t u) {
    const uint32_t n = 1u << u;
    for (uint32_t h = 1; h < n; h <<= 1) {
        for (uint32_t k = threadIdx.x; k < n / 2; k += blockDim.x) {
            const uint32_t i = (k / h) * 2 * h + (k % h);
            const uint32_t p = v[i], q = v[i + h];
            v[i] = add_mod(p, q);
            v[i + h] = sub_mod(p, q);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(1024) k_eval_poly(uint32_t u, uint32_t low_rate, uint32_t end, const uint8_t *state,
                                                    const uint16_t *lw_fold, uint32_t lw0, uint32_t *rowinfo) {
    extern __shared__ __attribute__((aligned(16))) uint16_t v[];
    const uint32_t n = 1u << u;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t e = state[i] & 1u;
        // high rate: v = e;  low rate: v = e - 1 on [0, end), 0 beyond  (mod 65535)
        v[i] = low_rate ? (i < end ? (e ? 0u : 65534u) : 0u) : e;
    }
    __syncthreads();
    walsh_lds(v, u);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t p = uint32_t(v[i]) * lw_fold[i];
        uint32_t f = add_mod(p & 0xFFFFu, p >> 16);
        if (low_rate && i == 0) f = add_mod(f, lw0);
        v[i] = f;
    }
    __syncthreads();
    walsh_lds(v, u);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
        rowinfo[i] = v[i] | ((state[i] & 2u) ? 0u : 0x10000u);
}

__global__ void k_mul(uint8_t *rows, uint64_t packs, const uint32_t *t) {
    const uint64_t pk = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (pk >= packs) return;
    uint32_t *p = reinterpret_cast<uint32_t *>(rows + (pk >> 3) * 64 + (pk & 7) * 4);
    uint32_t l = p[0], h = p[8];
    gf_mul4(l, h, t);
    p[0] = l;
    p[8] = h;
}

__global__ void k_formal_derivative(const uint8_t *in, uint8_t *out, uint32_t rows, uint64_t words_per_row) {
    const uint64_t wi = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint32_t q = blockIdx.y;
    if (wi >= words_per_row) return;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(in);
    uint32_t acc = src[uint64_t(q) * words_per_row + wi];
    for (uint32_t b = 1; b < rows; b <<= 1)
        if (!(q & b) && (q | b) < rows) acc ^= src[uint64_t(q | b) * words_per_row + wi];
    reinterpret_cast<uint32_t *>(out)[uint64_t(q) * words_per_row + wi] = acc;
}

}  // namespace

hipError_t launch_pass(int K, int flags, const PassArgs &A, hipStream_t s) {
    switch (K) {
        case 0: return launch_k<0, 0>(flags, A, s);
        case 1: return launch_k<1, 1>(flags, A, s);
        case 2: return launch_k<2, 1>(flags, A, s);
        case 3: return launch_k<3, 2>(flags, A, s);
        case 4: return launch_k<4, 2>(flags, A, s);
        case 5: return launch_k<5, 3>(flags, A, s);
        case 6: return launch_k<6, 3>(flags, A, s);
        case 7: return launch_k<7, 4>(flags, A, s);
        case 8: return launch_k<8, 4>(flags, A, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_eval_poly(uint32_t u, bool low_rate, uint32_t end, const uint8_t *state, const uint16_t *lw_fold_u,
                            uint16_t log_walsh0, uint32_t *rowinfo, hipStream_t s) {
    const size_t lds = size_t(2) << u;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_eval_poly),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 2 << 16);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    k_eval_poly<<<1, 1024, lds, s>>>(u, low_rate ? 1u : 0u, end, state, lw_fold_u, log_walsh0, rowinfo);
    return hipGetLastError();
}

hipError_t launch_mul(uint8_t *rows, uint64_t blocks, const uint32_t *t, hipStream_t s) {
    const uint64_t packs = blocks * 8;
    if (!packs) return hipSuccess;
    k_mul<<<dim3(uint32_t((packs + 255) / 256)), 256, 0, s>>>(rows, packs, t);
    return hipGetLastError();
}

hipError_t launch_formal_derivative(const uint8_t *in, uint8_t *out, uint32_t rows, uint64_t row_bytes, hipStream_t s) {
    const uint64_t words = row_bytes / 4;
    if (!rows || !words) return hipSuccess;
    k_formal_derivative<<<dim3(uint32_t((words + 255) / 256), rows), 256, 0, s>>>(in, out, rows, words);
    return hipGetLastError();
}

}  // namespace rs
