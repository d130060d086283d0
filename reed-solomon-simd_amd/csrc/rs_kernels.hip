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
        // '+' (not '|': the bits are disjoint) lets the compiler fold the
        // register index into LDS / global immediate offsets
        if constexpr (W == 1) return i;
        if constexpr (PB) return (uint32_t(i) << (K - LR)) + w;
        return (w << LR) + uint32_t(i);
    }
};

struct Ctx {
    uint32_t lane, w, s_lo, s_hi, a, pk_off;
    bool pk_ok;
    __device__ __forceinline__ uint32_t grow(uint32_t j, int K) const { return s_lo + (j << a) + (s_hi << (a + K)); }
};

// LDS layout (dynamic, 16-byte aligned), in 32-bit words:
//   plane : 64 lanes x 2^K rows, one data plane (low or high words) at a time
//   tab   : 2^K tables x 20 words -- the twiddle tables of the transform in
//           flight (slot = 2^K - 2^(K-b) + group, b = local layer), or the
//           per-row scale tables of a decode load / reveal
//   rinfo : 2^K words -- decode row info of the set's rows
template <int K>
struct Lds {
    static constexpr uint32_t kPlane = uint32_t(kLanes) << K;
    static constexpr uint32_t kTab = 20u << K;
    static constexpr uint32_t kRows = 1u << K;
    static constexpr size_t bytes() { return size_t(kPlane + kTab + kRows) * 4; }
};

// slot of the twiddle table of local layer b for local row j (bit b of j clear)
template <int K>
__device__ __forceinline__ uint32_t tw_slot(int b, uint32_t j) {
    return (1u << K) - (1u << (K - b)) + (j >> (b + 1));
}

// Stage the 2^K - 1 twiddle tables of this set for one transform into LDS.
template <int K>
__device__ __forceinline__ void stage_twiddles(const PassArgs &A, const Ctx &c, uint32_t delta, uint32_t *tab) {
    constexpr uint32_t slots = (1u << K) - 1;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < slots * 20; t += blockDim.x) {
        const uint32_t slot = t / 20, word = t - slot * 20;
        const uint32_t y = (1u << K) - slot;                  // in [2, 2^K]
        const int b = K - (32 - __builtin_clz(y - 1));        // K - ceil(log2 y)
        const uint32_t g = slot - ((1u << K) - (1u << (K - b)));
        const uint32_t row = c.grow(g << (b + 1), K);
        const uint32_t gb = c.a + b;
        const uint32_t idx = (row & ~((2u << gb) - 1u)) + (1u << gb) + delta - 1u;
        tab[t] = A.tw[idx * 20u + word];
    }
    __syncthreads();
}

// Stage per-row decode info and scale tables (load: factor, reveal: 65535 - factor).
template <int K>
__device__ __forceinline__ void stage_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, bool reveal,
                                           uint32_t *tab, uint32_t *rinfo) {
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < (1u << K); t += blockDim.x) rinfo[t] = A.rowinfo[c.grow(t, K) + chunk * A.n];
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < (20u << K); t += blockDim.x) {
        const uint32_t j = t / 20, word = t - j * 20;
        const uint32_t f = rinfo[j] & 0xFFFFu;
        tab[t] = A.lut[(reveal ? 65535u - f : f) * 20u + word];
    }
    __syncthreads();
}

template <int K, int LR, bool PB, bool SCALE>
__device__ __forceinline__ void load_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, const uint32_t *tab,
                                          const uint32_t *rinfo, uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<PB>(c.w, i);
        uint32_t r = c.grow(j, K) + chunk * A.n;
        r = __builtin_amdgcn_readfirstlane(r);
        asm volatile("" : "+s"(r));  // keep the row's address math here, not hoisted
        const uint8_t *p = nullptr;
        if (A.work_in) {
            p = A.work_in + uint64_t(r) * A.work_stride;
        } else {
            if (r >= A.src[0].row_begin && r < A.src[0].row_end)
                p = A.src[0].base + uint64_t(r - A.src[0].row_begin) * A.src[0].stride;
            if (A.nsrc > 1 && r >= A.src[1].row_begin && r < A.src[1].row_end)
                p = A.src[1].base + uint64_t(r - A.src[1].row_begin) * A.src[1].stride;
        }
        if (SCALE && (rinfo[j] & 0x10000u)) p = nullptr;
        uint32_t l = 0, h = 0;
        if (p && c.pk_ok) {
            l = *reinterpret_cast<const uint32_t *>(p + c.pk_off);
            h = *reinterpret_cast<const uint32_t *>(p + c.pk_off + 32);
        }
        lo[i] = l;
        hi[i] = h;
    });
    if constexpr (SCALE) {
        uint32_t dep = 0;
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            uint32_t off = P::template lrow<PB>(c.w, i) * 20u;
            asm volatile("" : "+s"(off), "+v"(lo[i]), "+v"(hi[i]) : "v"(dep));  // one row at a time
            gf_mul4(lo[i], hi[i], tab + off);
            dep = lo[i];
        });
    }
}

template <int K, int LR, bool PB, bool REVEAL>
__device__ __forceinline__ void store_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, const uint32_t *tab,
                                           const uint32_t *rinfo, uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<PB>(c.w, i);
        uint32_t r = c.grow(j, K) + chunk * A.n;
        r = __builtin_amdgcn_readfirstlane(r);
        asm volatile("" : "+s"(r));  // keep the row's address math here, not hoisted
        uint8_t *p = nullptr;
        uint32_t l = lo[i], h = hi[i];
        if (A.work_out) {
            p = A.work_out + uint64_t(r) * A.work_stride;
        } else if (r >= A.dst.row_begin && r < A.dst.row_end) {
            p = const_cast<uint8_t *>(A.dst.base) + uint64_t(r - A.dst.row_begin) * A.dst.stride;
            if constexpr (REVEAL) {
                if (rinfo[j] & 0x10000u) gf_mul4(l, h, tab + j * 20u);
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
__device__ __forceinline__ void layer(const Ctx &c, const uint32_t *tab, uint32_t (&lo)[1 << LR],
                                      uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    constexpr int RB = PB && P::W > 1 ? B - (K - LR) : B;  // register bit
    static_assert(RB >= 0 && RB < LR, "bit not resident in this phase");
    // Butterfly groups of this layer held by the lane: register index bits
    // above RB.  One 20-word table per group, read from LDS once and used for
    // the group's 2^RB butterflies.  The table's address is tied (empty asm)
    // to the previous group's result, so at most one table is in flight:
    // otherwise the compiler hoists every table of the layer and spills.
    uint32_t dep = 0;
    static_for<0, (P::R >> (RB + 1))>([&](auto gc) {
        constexpr int i0 = decltype(gc)::value << (RB + 1);
        uint32_t off = tw_slot<K>(B, P::template lrow<PB>(c.w, i0)) * 20u;
        asm volatile("" : "+s"(off) : "v"(dep));
        const uint4 *t4 = reinterpret_cast<const uint4 *>(tab + off);
        uint32_t t[20];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint4 v = t4[q];
            t[4 * q] = v.x, t[4 * q + 1] = v.y, t[4 * q + 2] = v.z, t[4 * q + 3] = v.w;
        }
        static_for<0, (1 << RB)>([&](auto lc) {
            constexpr int i = i0 | decltype(lc)::value;
            constexpr int i2 = i | (1 << RB);
            // The butterflies are independent; left alone the compiler
            // interleaves all of them (~18 live VGPRs each) and spills.  Tie
            // each one's inputs to the previous one's output: one butterfly
            // in flight per wave, the other waves of the SIMD fill the gaps.
            asm volatile("" : "+v"(lo[i]), "+v"(hi[i]), "+v"(lo[i2]), "+v"(hi[i2]) : "v"(dep));
            if constexpr (IFFT) ifft_bfly(lo[i], hi[i], lo[i2], hi[i2], t);
            else fft_bfly(lo[i], hi[i], lo[i2], hi[i2], t);
            dep = lo[i];
        });
    });
}

// Move the rows from phase FROM_B to phase TO_B through LDS, one plane at a time.
template <int K, int LR, bool FROM_B, bool TO_B>
__device__ __forceinline__ void exchange(const Ctx &c, uint32_t *plane, uint32_t (&lo)[1 << LR],
                                         uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    if constexpr (P::W == 1 || FROM_B == TO_B) return;
    auto one = [&](uint32_t(&v)[1 << LR]) {
        __syncthreads();
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            plane[P::template lrow<FROM_B>(c.w, i) * kLanes + c.lane] = v[i];
        });
        __syncthreads();
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            v[i] = plane[P::template lrow<TO_B>(c.w, i) * kLanes + c.lane];
        });
    };
    one(lo);
    one(hi);
}

// Formal derivative restricted to the set's local bits, plane by plane:
//   x[q] <- (mode 2 ? x[q] : 0) ^ XOR_{b < K, q_b = 0} x[q | 2^b]
template <int K, int LR, bool PB>
__device__ __forceinline__ void formal_derivative(const Ctx &c, uint32_t mode, uint32_t *plane,
                                                  uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    auto one = [&](uint32_t(&v)[1 << LR]) {
        __syncthreads();
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            plane[P::template lrow<PB>(c.w, i) * kLanes + c.lane] = v[i];
        });
        __syncthreads();
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const uint32_t j = P::template lrow<PB>(c.w, i);
            uint32_t acc = mode == 2 ? v[i] : 0u;
#pragma unroll
            for (int b = 0; b < K; ++b)
                if (!(j & (1u << b))) acc ^= plane[(j | (1u << b)) * kLanes + c.lane];
            v[i] = acc;
            asm volatile("" ::: "memory");
        });
    };
    one(lo);
    one(hi);
}

template <int K, int LR, bool PB>
__device__ __forceinline__ void xor_rows_in(const PassArgs &A, const Ctx &c, uint32_t (&lo)[1 << LR],
                                            uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        uint32_t r = c.grow(P::template lrow<PB>(c.w, i), K);
        r = __builtin_amdgcn_readfirstlane(r);
        asm volatile("" : "+s"(r));
        const uint8_t *p = A.xor_in + uint64_t(r) * A.work_stride;
        if (c.pk_ok) {
            lo[i] ^= *reinterpret_cast<const uint32_t *>(p + c.pk_off);
            hi[i] ^= *reinterpret_cast<const uint32_t *>(p + c.pk_off + 32);
        }
    });
}

template <int K, int LR, bool IFFT>
__device__ __forceinline__ void transform(const Ctx &c, uint32_t *plane, const uint32_t *tab,
                                          uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR>;
    constexpr bool HAS_B = P::W > 1;
    if constexpr (IFFT) {  // bits ascending: A-phase [0, LR), B-phase [LR, K)
        static_for<0, (LR < K ? LR : K)>([&](auto bc) { layer<K, LR, false, decltype(bc)::value, true>(c, tab, lo, hi); });
        if constexpr (HAS_B) {
            exchange<K, LR, false, true>(c, plane, lo, hi);
            static_for<LR, K>([&](auto bc) { layer<K, LR, true, decltype(bc)::value, true>(c, tab, lo, hi); });
        }
    } else {  // bits descending: B-phase [LR, K), A-phase [0, LR)
        if constexpr (HAS_B) {
            static_for<0, K - LR>([&](auto bc) { layer<K, LR, true, K - 1 - decltype(bc)::value, false>(c, tab, lo, hi); });
            exchange<K, LR, true, false>(c, plane, lo, hi);
        }
        static_for<0, (LR < K ? LR : K)>([&](auto bc) {
            constexpr int b = (LR < K ? LR : K) - 1 - decltype(bc)::value;
            layer<K, LR, false, b, false>(c, tab, lo, hi);
        });
    }
}

template <int K, int LR, int FLAGS>
__global__ void __launch_bounds__(kLanes << (K - LR), 2) k_pass(const PassArgs A) {
    using P = Pass<K, LR>;
    constexpr bool DO_IFFT = FLAGS & kIfft;
    constexpr bool DO_FFT = FLAGS & kFft;
    constexpr bool MULTI_IN = FLAGS & kMultiIn;    // XOR-fold IFFTs of A.in_chunks chunks
    constexpr bool MULTI_OUT = FLAGS & kMultiOut;  // FFT the same rows for A.out_chunks chunks
    constexpr bool SCALE = FLAGS & kScale;         // decode: scale received rows, zero erased ones
    constexpr bool FD = FLAGS & kFd;               // decode: formal derivative over local bits
    constexpr bool XOR_IN = FLAGS & kXorIn;        // decode: x ^= rows of A.xor_in
    constexpr bool REVEAL = FLAGS & kReveal;       // decode: store erased originals, unscaled
    constexpr bool HAS_B = P::W > 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t *plane = lds;
    uint32_t *tab = lds + Lds<K>::kPlane;
    uint32_t *rinfo = tab + Lds<K>::kTab;

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
    if constexpr (DO_IFFT && !MULTI_IN) {
        if constexpr (SCALE) stage_rows<K>(A, c, gchunk, false, tab, rinfo);
        load_rows<K, LR, false, SCALE>(A, c, gchunk, tab, rinfo, lo, hi);
        if constexpr (K > 0) stage_twiddles<K>(A, c, A.ifft_delta + gchunk * A.ifft_delta_step, tab);
        transform<K, LR, true>(c, plane, tab, lo, hi);
    } else if constexpr (DO_IFFT) {
        uint32_t tl[P::R], th[P::R];
        for (uint32_t ci = 0; ci < A.in_chunks; ++ci) {
            const uint32_t chunk = gchunk + ci;
            if constexpr (SCALE) stage_rows<K>(A, c, chunk, false, tab, rinfo);
            load_rows<K, LR, false, SCALE>(A, c, chunk, tab, rinfo, tl, th);
            if constexpr (K > 0) stage_twiddles<K>(A, c, A.ifft_delta + chunk * A.ifft_delta_step, tab);
            transform<K, LR, true>(c, plane, tab, tl, th);
            if (ci == 0) {
                static_for<0, P::R>([&](auto ic) { lo[ic] = tl[ic]; hi[ic] = th[ic]; });
            } else {
                static_for<0, P::R>([&](auto ic) { lo[ic] ^= tl[ic]; hi[ic] ^= th[ic]; });
            }
        }
    } else {
        if constexpr (SCALE) stage_rows<K>(A, c, gchunk, false, tab, rinfo);
        load_rows<K, LR, HAS_B, SCALE>(A, c, gchunk, tab, rinfo, lo, hi);
    }
    // rows are now in phase B (if the pass has one)

    if constexpr (FD) formal_derivative<K, LR, HAS_B>(c, A.fd_mode, plane, lo, hi);
    if constexpr (XOR_IN) xor_rows_in<K, LR, HAS_B>(A, c, lo, hi);

    // ---- FFT per output chunk + store ------------------------------------
    if constexpr (DO_FFT && !MULTI_OUT) {
        if constexpr (K > 0) stage_twiddles<K>(A, c, A.fft_delta + gchunk * A.fft_delta_step, tab);
        transform<K, LR, false>(c, plane, tab, lo, hi);
        if constexpr (REVEAL) stage_rows<K>(A, c, gchunk, true, tab, rinfo);
        store_rows<K, LR, false, REVEAL>(A, c, gchunk, tab, rinfo, lo, hi);
    } else if constexpr (DO_FFT) {
        for (uint32_t co = 0; co < A.out_chunks; ++co) {
            const uint32_t chunk = gchunk + co;
            uint32_t yl[P::R], yh[P::R];
            static_for<0, P::R>([&](auto ic) { yl[ic] = lo[ic]; yh[ic] = hi[ic]; });
            if constexpr (K > 0) stage_twiddles<K>(A, c, A.fft_delta + chunk * A.fft_delta_step, tab);
            transform<K, LR, false>(c, plane, tab, yl, yh);
            if constexpr (REVEAL) stage_rows<K>(A, c, chunk, true, tab, rinfo);
            store_rows<K, LR, false, REVEAL>(A, c, chunk, tab, rinfo, yl, yh);
        }
    } else {
        if constexpr (REVEAL) stage_rows<K>(A, c, gchunk, true, tab, rinfo);
        store_rows<K, LR, HAS_B, REVEAL>(A, c, gchunk, tab, rinfo, lo, hi);
    }
}

template <int K, int LR, int F>
hipError_t launch_f(const PassArgs &A, hipStream_t s) {
    using P = Pass<K, LR>;
    const size_t lds = Lds<K>::bytes();
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
    if (A.in_chunks > 1) flags |= kMultiIn;
    if (A.out_chunks > 1) flags |= kMultiOut;
    if (A.load_scale) flags |= kScale;
    if (A.fd_mode) flags |= kFd;
    if (A.xor_in) flags |= kXorIn;
    if (A.reveal) flags |= kReveal;
    constexpr int I = kIfft, F = kFft;
    switch (flags) {
        // encode / engine
        case I: return launch_f<K, LR, I>(A, s);
        case F: return launch_f<K, LR, F>(A, s);
        case I | F: return launch_f<K, LR, I | F>(A, s);
        case I | kMultiIn: return launch_f<K, LR, I | kMultiIn>(A, s);
        case I | F | kMultiIn: return launch_f<K, LR, I | F | kMultiIn>(A, s);
        case I | F | kMultiOut: return launch_f<K, LR, I | F | kMultiOut>(A, s);
        case F | kMultiOut: return launch_f<K, LR, F | kMultiOut>(A, s);
        // decode: single pass, IFFT passes, fused top, FFT passes (middle / last)
        case I | F | kScale | kFd | kReveal: return launch_f<K, LR, I | F | kScale | kFd | kReveal>(A, s);
        case I | kScale: return launch_f<K, LR, I | kScale>(A, s);
        case I | F | kFd: return launch_f<K, LR, I | F | kFd>(A, s);
        case F | kFd | kXorIn: return launch_f<K, LR, F | kFd | kXorIn>(A, s);
        case F | kFd | kXorIn | kReveal: return launch_f<K, LR, F | kFd | kXorIn | kReveal>(A, s);
        default: return hipErrorInvalidValue;
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
