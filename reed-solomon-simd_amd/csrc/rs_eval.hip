// eval_poly of a decode on the device (reference src/engine/utils.rs:20-31,
// src/engine/fwht.rs:9-55) reduced to 2^u points: the erasure vector is zero
// outside [0, 2^u) for HighRate, and 1 there for LowRate (rate_low.rs:196),
// so FWHT_16 collapses onto 2^u residues: v -> FWHT_u -> x lw_fold -> FWHT_u
// (DESIGN.md "eval_poly").  All arithmetic is mod 65535; 0 and 65535 are the
// same residue and every consumer treats them alike.
//
// One workgroup of up to 1024 threads; one Walsh-Hadamard layer per barrier
// over LDS; every global read (bitmaps, folded log_walsh) is issued up front.
#include <hip/hip_runtime.h>

#include "rs_device.hpp"
#include "rs_gf.hpp"

namespace rs {
namespace {

#ifdef RS_EVAL_STAMPS  // tools/eval_probe.hip
__device__ uint64_t g_eval_stamps[8];
#define RS_ESTAMP(i)                                                      \
    do {                                                                  \
        __syncthreads();                                                  \
        if (threadIdx.x == 0) g_eval_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define RS_ESTAMP(i)
#endif

__device__ __forceinline__ uint32_t add_mod(uint32_t a, uint32_t b) {
    const uint32_t s = a + b;
    return (s + (s >> 16)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t sub_mod(uint32_t a, uint32_t b) {
    const uint32_t d = a - b;
    return (d + (d >> 16)) & 0xFFFFu;
}

// One Walsh-Hadamard layer per barrier on bit h of 2^u values in LDS: every
// thread takes the butterflies t, t + T, ... (pairs (i, i + 2^h)).
__device__ void walsh(uint16_t *v, uint32_t u) {
    const uint32_t half = 1u << (u - 1);
    for (uint32_t h = 0; h < u; ++h) {
        for (uint32_t k = threadIdx.x; k < half; k += blockDim.x) {
            const uint32_t i = ((k >> h) << (h + 1)) | (k & ((1u << h) - 1u));
            const uint32_t p = v[i], q = v[i + (1u << h)];
            v[i] = uint16_t(add_mod(p, q));
            v[i + (1u << h)] = uint16_t(sub_mod(p, q));
        }
        __syncthreads();
    }
}

// LDS: v[2^u] u16 values, then the erased / received bitmaps (2^u bits each).
__global__ void __launch_bounds__(1024) k_eval_poly(const EvalArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint16_t v[];
    const uint32_t n = 1u << A.u;
    const bool inl = n <= kEvalInlineRows;
    uint32_t *bits = reinterpret_cast<uint32_t *>(v + (n < 2 ? 2 : n));  // [0, nw): erased, [nw, 2nw): received
    const uint32_t nw = (n + 31) / 32;
    RS_ESTAMP(0);
    // every global read is issued up front: one memory latency, not one per phase
    uint32_t lw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t i = threadIdx.x + uint32_t(k) * blockDim.x;
        lw[k] = i < n ? A.lw_fold[i] : 0u;
    }
    if (inl) {
        for (uint32_t w = threadIdx.x; w < 2 * nw; w += blockDim.x)
            bits[w] = w < nw ? A.erased[w] : A.received[w - nw];
    } else {
        for (uint32_t w = threadIdx.x; w < 2 * nw; w += blockDim.x) {
            const uint32_t base = (w % nw) * 32, sh = w < nw ? 0 : 1;
            uint32_t x = 0;
            for (uint32_t j = 0; j < 32 && base + j < n; ++j) x |= ((A.state[base + j] >> sh) & 1u) << j;
            bits[w] = x;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t e = (bits[i >> 5] >> (i & 31)) & 1u;
        // high rate: v = e;  low rate: v = e - 1 on [0, end), 0 beyond  (mod 65535)
        v[i] = uint16_t(A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e);
    }
    __syncthreads();
    RS_ESTAMP(1);
    walsh(v, A.u);
    RS_ESTAMP(2);
    for (uint32_t i = threadIdx.x, k = 0; i < n; i += blockDim.x, ++k) {
        const uint32_t p = uint32_t(v[i]) * (k < 8 ? lw[k & 7] : A.lw_fold[i]);
        uint32_t f = add_mod(p & 0xFFFFu, p >> 16);
        if (A.low_rate && i == 0) f = add_mod(f, A.lw0);
        v[i] = uint16_t(f);
    }
    __syncthreads();
    RS_ESTAMP(3);
    walsh(v, A.u);
    RS_ESTAMP(4);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t rcv = (bits[nw + (i >> 5)] >> (i & 31)) & 1u;
        A.rowinfo[i] = v[i] | (rcv ? 0u : 0x10000u);
    }
    RS_ESTAMP(5);
}

// 2^11 .. 2^13 points (pass-kernel decodes of 2048 .. 8192 work rows): one
// workgroup of 1024 threads, thread t holding rows t*V .. t*V + V - 1
// (V = 2^(u - 10)), the transform as in the column kernel's fused eval_poly
// (rs_mono.hip col_walsh): log2(V) layers in registers, 6 across lanes by DPP /
// v_permlane*_swap, the 4 wave bits as two LDS rounds of two layers, lazy
// reduction mod 65535 (values below B_k after k layers, folded at the end).
// It replaces 22 one-layer barriers (2^11: 8.2 -> 3.2..5.0 us per launch) or
// three launches (2^12: 10.0 -> 5.0 us, 2^13: 10.6 -> 8.3 us; tools/eval_probe.hip,
// profiles/r03b, profiles/r04a).
constexpr uint64_t ev_bound(int k) {  // B_k: values stay below it after k lazy layers
    uint64_t b = 65536u;
    for (int i = 0; i < k; ++i) b = 2 * b + 65535u;
    return b;
}
template <int K>  // M_K + 1, M_K the least multiple of 65535 >= B_K
constexpr uint32_t kEvM1 = uint32_t((ev_bound(K) + 65534u) / 65535u * 65535u) + 1u;
static_assert(ev_bound(13) < (1ull << 32), "lazy Walsh-Hadamard bound at 2^13 points");
__device__ __forceinline__ uint32_t ev_fold(uint32_t x) {
    x = (x & 0xFFFFu) + (x >> 16);
    return (x & 0xFFFFu) + (x >> 16);
}

// The LDS rounds keep value v of thread t at word v * 1024 + t: a wave's
// stores and reads are 64 consecutive words.  (Thread-major, t * V + v, is a
// V-way bank conflict: 2^13 points 10.65 -> 8.27 us, 2^12 5.02 -> 4.87 us per
// launch, profiles/r04a/eval_vmajor_ab.txt; RS_EVAL_VMAJOR=0 for the A/B.)
#ifndef RS_EVAL_VMAJOR
#define RS_EVAL_VMAJOR 1
#endif
// One 2^(LV + 10)-point transform; G0: index of its first LDS round (rounds
// alternate the two buffers across both transforms, so no barrier between them)
template <int LV, int G0>
__device__ __forceinline__ void walsh_fast(uint32_t (&x)[1 << LV], uint32_t *buf) {
    constexpr int V = 1 << LV, L = LV + 10;
    const uint32_t t = threadIdx.x, lane = t & 63u;
    // LDS word of value v of thread q
    auto ix = [](uint32_t q, int v) { return RS_EVAL_VMAJOR ? uint32_t(v) * 1024u + q : q * V + uint32_t(v); };
    static_for<0, LV>([&](auto kc) {  // register bits
        constexpr int k = decltype(kc)::value;
        static_for<0, V>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            if constexpr (!(v & (1 << k))) {
                const uint32_t a = x[v], b = x[v | (1 << k)];
                x[v] = a + b;
                x[v | (1 << k)] = a + ~b + kEvM1<k>;
            }
        });
    });
    static_for<0, 6>([&](auto jc) {  // lane bits
        constexpr int J = decltype(jc)::value;
        const uint32_t m = (lane & (1u << J)) ? ~0u : 0u, c = m & kEvM1<LV + J>;
        static_for<0, V>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            x[v] = lane_xor<J>(x[v], lane) + (x[v] ^ m) + c;
        });
    });
    static_for<0, 2>([&](auto rc) {  // wave bits: thread bits 6 + 2 rnd, 7 + 2 rnd
        constexpr int rnd = decltype(rc)::value;
        constexpr int j = LV + 6 + 2 * rnd;  // layers j, j + 1
        constexpr uint32_t h1 = 64u << (2 * rnd), h2 = h1 << 1;
        uint32_t *b = buf + ((((G0 + rnd) & 1) ^ 1) << L);
        static_for<0, V>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            b[ix(t, v)] = x[v];
        });
        __syncthreads();
        const uint32_t m1 = (t & h1) ? ~0u : 0u, c1 = m1 & kEvM1<j>;
        const uint32_t m2 = (t & h2) ? ~0u : 0u, c2 = m2 & kEvM1<j + 1>;
        const uint32_t g0 = t & ~(h1 | h2);
        static_for<0, V>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const uint32_t v00 = b[ix(g0, v)], v01 = b[ix(g0 | h1, v)];
            const uint32_t v10 = b[ix(g0 | h2, v)], v11 = b[ix(g0 | h1 | h2, v)];
            const uint32_t lo = v00 + (v01 ^ m1) + c1, hi = v10 + (v11 ^ m1) + c1;
            x[v] = lo + (hi ^ m2) + c2;
        });
    });
    static_for<0, V>([&](auto vc) { x[decltype(vc)::value] = ev_fold(x[decltype(vc)::value]); });
}

template <int LV>
__global__ void __launch_bounds__(1024) k_eval_fast(const EvalArgs A) {
    constexpr int V = 1 << LV;
    extern __shared__ __attribute__((aligned(16))) uint32_t ebuf[];  // 2 x 2^(LV + 10) words
    const uint32_t r0 = threadIdx.x * V;
    uint32_t lw[V], x[V];
    static_for<0, V>([&](auto vc) { lw[decltype(vc)::value] = A.lw_fold[r0 + decltype(vc)::value]; });
    // V consecutive rows lie in one bitmap word (inline bitmaps: 2^u <= kEvalInlineRows)
    const uint32_t eb = A.erased[r0 >> 5] >> (r0 & 31u), rb = A.received[r0 >> 5] >> (r0 & 31u);
    static_for<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const uint32_t e = (eb >> v) & 1u, i = r0 + v;
        // high rate: v = e;  low rate: v = e - 1 on [0, end), 0 beyond  (rate_low.rs:196)
        x[v] = A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e;
    });
    walsh_fast<LV, 0>(x, ebuf);
    static_for<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const uint32_t p = x[v] * lw[v];
        uint32_t f = add_mod(p & 0xFFFFu, p >> 16);
        if (A.low_rate && r0 + v == 0) f = add_mod(f, A.lw0);
        x[v] = f;
    });
    walsh_fast<LV, 2>(x, ebuf);
    static_for<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        A.rowinfo[r0 + v] = x[v] | (((rb >> v) & 1u) ? 0u : 0x10000u);
    });
}
#ifndef RS_EVAL_FAST_MIN_U  // (A/B: 14 = off)
#define RS_EVAL_FAST_MIN_U 11
#endif
#ifndef RS_EVAL_FAST_MAX_U  // (A/B: 12 = 2^13 points on the three-launch form)
#define RS_EVAL_FAST_MAX_U 13
#endif

// Large transforms (2^u > kEvalSingleRows) spread over many workgroups: the
// two FWHT_u split into their low bits [0, K1) and high bits [K1, u), four
// launches, one workgroup per set of 2^K values that differ only in those
// bits (Walsh-Hadamard layers on different bits commute).  The values live in
// `rowinfo` (u32) between launches.
//   STEP 0: values from the erasure state, low bits
//   STEP 1: high bits, then x lw_fold (+ log_walsh[0] at 0 for low rate)
//   STEP 2: low bits
//   STEP 3: high bits, then rowinfo = value | not-received bit
constexpr uint32_t kEvalSingleRows = 2048;

__device__ __forceinline__ uint32_t state_bit(const EvalArgs &A, uint32_t i, uint32_t which) {
    if ((1u << A.u) <= kEvalInlineRows) return ((which ? A.received : A.erased)[i >> 5] >> (i & 31)) & 1u;
    return (A.state[i] >> which) & 1u;
}

template <int STEP>
__global__ void __launch_bounds__(512) k_walsh_part(const EvalArgs A, uint32_t a, uint32_t K) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sv[];
    const uint32_t m = 1u << K, set = blockIdx.x;
    const uint32_t lo = set & ((1u << a) - 1u), hi = set >> a;
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
        const uint32_t i = lo + (j << a) + (hi << (a + K));
        uint32_t x;
        if constexpr (STEP == 0) {
            const uint32_t e = state_bit(A, i, 0);
            x = A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e;
        } else {
            x = A.rowinfo[i];
        }
        sv[j] = x;
    }
    __syncthreads();
    const auto walsh = [&]() {
        for (uint32_t h = 0; h < K; ++h) {
            for (uint32_t k = threadIdx.x; k < m / 2; k += blockDim.x) {
                const uint32_t i = ((k >> h) << (h + 1)) | (k & ((1u << h) - 1u));
                const uint32_t p = sv[i], q = sv[i + (1u << h)];
                sv[i] = add_mod(p, q);
                sv[i + (1u << h)] = sub_mod(p, q);
            }
            __syncthreads();
        }
    };
    walsh();
    if constexpr (STEP == 1) {  // x lw_fold between the two transforms' high-bit layers
        for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
            const uint32_t i = lo + (j << a) + (hi << (a + K));
            const uint32_t p = sv[j] * A.lw_fold[i];
            uint32_t x = add_mod(p & 0xFFFFu, p >> 16);
            if (A.low_rate && i == 0) x = add_mod(x, A.lw0);
            sv[j] = x;
        }
        __syncthreads();
        walsh();
    }
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
        const uint32_t i = lo + (j << a) + (hi << (a + K));
        uint32_t x = sv[j];
        if constexpr (STEP == 3) x |= state_bit(A, i, 1) ? 0u : 0x10000u;
        A.rowinfo[i] = x;
    }
}

// The same steps with one wave per set of 2^K values (K = 7, 8): lane l holds
// values j = l * V .. l * V + V - 1 (V = 2^(K - 6)); the log2(V) low layers in
// registers, the 6 above across lanes by DPP / permlane swaps -- no LDS and no
// barrier (k_walsh_part: one layer per barrier).  Layers run in the same order,
// each exact mod 65535 (add_mod / sub_mod), so the values are identical.
template <int STEP, int K>
__global__ void __launch_bounds__(64) k_walsh_wave(const EvalArgs A, uint32_t a) {
    constexpr int LV = K - 6, V = 1 << LV;
    const uint32_t set = blockIdx.x, lane = threadIdx.x;
    const uint32_t lo = set & ((1u << a) - 1u), hi = set >> a;
    auto row = [&](int v) { return lo + ((lane * V + uint32_t(v)) << a) + (hi << (a + K)); };
    uint32_t x[V];
    static_for<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const uint32_t i = row(v);
        if constexpr (STEP == 0) {
            const uint32_t e = state_bit(A, i, 0);
            x[v] = A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e;
        } else {
            x[v] = A.rowinfo[i];
        }
    });
    auto walsh = [&]() {
        static_for<0, LV>([&](auto hc) {  // register bits
            constexpr int h = decltype(hc)::value;
            static_for<0, V>([&](auto vc) {
                constexpr int v = decltype(vc)::value;
                if constexpr (!(v & (1 << h))) {
                    const uint32_t p = x[v], q = x[v | (1 << h)];
                    x[v] = add_mod(p, q);
                    x[v | (1 << h)] = sub_mod(p, q);
                }
            });
        });
        static_for<0, 6>([&](auto jc) {  // lane bits
            constexpr int J = decltype(jc)::value;
            static_for<0, V>([&](auto vc) {
                constexpr int v = decltype(vc)::value;
                const uint32_t o = lane_xor<J>(x[v], lane);
                x[v] = (lane >> J) & 1u ? sub_mod(o, x[v]) : add_mod(x[v], o);
            });
        });
    };
    walsh();
    if constexpr (STEP == 1) {  // x lw_fold between the two transforms' high-bit layers
        static_for<0, V>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const uint32_t i = row(v);
            const uint32_t p = x[v] * A.lw_fold[i];
            uint32_t f = add_mod(p & 0xFFFFu, p >> 16);
            if (A.low_rate && i == 0) f = add_mod(f, A.lw0);
            x[v] = f;
        });
        walsh();
    }
    static_for<0, V>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        const uint32_t i = row(v);
        uint32_t y = x[v];
        if constexpr (STEP == 3) y |= state_bit(A, i, 1) ? 0u : 0x10000u;
        A.rowinfo[i] = y;
    });
}

#ifndef RS_EVAL_WAVE  // (A/B: 0 = k_walsh_part, one layer per barrier)
#define RS_EVAL_WAVE 1
#endif
template <int STEP>
void walsh_step(const EvalArgs &A, uint32_t a, uint32_t K, uint32_t n, hipStream_t s) {
    if (RS_EVAL_WAVE && K == 7) {
        k_walsh_wave<STEP, 7><<<n >> 7, 64, 0, s>>>(A, a);
    } else if (RS_EVAL_WAVE && K == 8) {
        k_walsh_wave<STEP, 8><<<n >> 8, 64, 0, s>>>(A, a);
    } else {
        const uint32_t m = 1u << K;
        k_walsh_part<STEP><<<n >> K, m / 2 < 64 ? 64 : (m / 2 > 512 ? 512 : m / 2), size_t(4) * m, s>>>(A, a, K);
    }
}

}  // namespace

hipError_t launch_eval_poly(const EvalArgs &A, hipStream_t s) {
    const uint32_t n = 1u << A.u;
    // (2^13 points: 8.3 us in one workgroup against 10.6 us in three launches)
    if (A.u >= RS_EVAL_FAST_MIN_U && A.u <= RS_EVAL_FAST_MAX_U) {
        static_assert((1u << 13) <= kEvalInlineRows, "k_eval_fast reads the inline bitmaps");
        const size_t lds = size_t(8) * n;  // two exchange buffers of 2^u words
        static std::atomic<uint64_t> fast_devs[3] = {{0}, {0}, {0}};  // per kernel: devices set
        const void *kf[3] = {reinterpret_cast<const void *>(&k_eval_fast<1>),
                             reinterpret_cast<const void *>(&k_eval_fast<2>),
                             reinterpret_cast<const void *>(&k_eval_fast<3>)};
        for (int k = 0; k < 3; ++k) {
            hipError_t e = lds_attr_once(fast_devs[k], kf[k], 64 * 1024);
            if (e != hipSuccess) return e;
        }
        if (A.u == 11) k_eval_fast<1><<<1, 1024, lds, s>>>(A);
        else if (A.u == 12) k_eval_fast<2><<<1, 1024, lds, s>>>(A);
        else k_eval_fast<3><<<1, 1024, lds, s>>>(A);
        return hipGetLastError();
    }
    if (n > kEvalSingleRows) {
        const uint32_t K1 = A.u / 2, K2 = A.u - K1;
        // Walsh-Hadamard layers on different bits commute: low bits of the
        // first transform; high bits of both around the multiply (one launch);
        // low bits of the second transform + output
        walsh_step<0>(A, 0, K1, n, s);
        walsh_step<1>(A, K1, K2, n, s);
        walsh_step<3>(A, 0, K1, n, s);
        return hipGetLastError();
    }
    const size_t lds = size_t(2) * (n < 2 ? 2 : n) + size_t(8) * ((n + 31) / 32);
    static std::atomic<uint64_t> attr_devs{0};  // devices whose attribute is set
    {
        hipError_t e = lds_attr_once(attr_devs, reinterpret_cast<const void *>(&k_eval_poly), 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const uint32_t threads = n / 2 >= 1024 ? 1024 : (n / 2 < 64 ? 64 : n / 2);
    k_eval_poly<<<1, threads, lds, s>>>(A);
    return hipGetLastError();
}

}  // namespace rs
