// eval_poly of a decode on the device (reference src/engine/utils.rs:20-31,
// src/engine/fwht.rs:9-55) reduced to 2^u points: the erasure vector is zero
// outside [0, 2^u) for HighRate, and 1 there for LowRate (rate_low.rs:196),
// so FWHT_16 collapses onto 2^u residues: v -> FWHT_u -> x lw_fold -> FWHT_u
// (DESIGN.md "eval_poly").  All arithmetic is mod 65535; 0 and 65535 are the
// same residue and every consumer treats them alike.
//
// One workgroup; the Walsh-Hadamard layers run 3 at a time in registers
// (8 values per thread per round), rounds meet in LDS.
#include <hip/hip_runtime.h>

#include "rs_device.hpp"

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

// Q layers of the transform on bits [a, a + Q) for every group of 2^Q values.
template <int Q>
__device__ __forceinline__ void walsh_round(uint16_t *v, uint32_t u, uint32_t a) {
    const uint32_t groups = 1u << (u - Q);
    for (uint32_t g = threadIdx.x; g < groups; g += blockDim.x) {
        const uint32_t base = (g & ((1u << a) - 1u)) | ((g >> a) << (a + Q));
        uint32_t x[1 << Q];
#pragma unroll
        for (int j = 0; j < (1 << Q); ++j) x[j] = v[base + (uint32_t(j) << a)];
#pragma unroll
        for (int l = 0; l < Q; ++l)
#pragma unroll
            for (int j = 0; j < (1 << Q); ++j)
                if (!(j & (1 << l))) {
                    const uint32_t p = x[j], q = x[j | (1 << l)];
                    x[j] = add_mod(p, q);
                    x[j | (1 << l)] = sub_mod(p, q);
                }
#pragma unroll
        for (int j = 0; j < (1 << Q); ++j) v[base + (uint32_t(j) << a)] = uint16_t(x[j]);
    }
    __syncthreads();
}

__device__ void walsh(uint16_t *v, uint32_t u) {
    uint32_t a = 0;
    for (; a + 3 <= u; a += 3) walsh_round<3>(v, u, a);
    if (u - a == 2) walsh_round<2>(v, u, a);
    else if (u - a == 1) walsh_round<1>(v, u, a);
}

__global__ void __launch_bounds__(1024) k_eval_poly(const EvalArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint16_t v[];
    const uint32_t n = 1u << A.u;
    const bool inl = n <= kEvalInlineRows;
    RS_ESTAMP(0);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t e = inl ? (A.erased[i >> 5] >> (i & 31)) & 1u : A.state[i] & 1u;
        // high rate: v = e;  low rate: v = e - 1 on [0, end), 0 beyond  (mod 65535)
        v[i] = uint16_t(A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e);
    }
    __syncthreads();
    RS_ESTAMP(1);
    walsh(v, A.u);
    RS_ESTAMP(2);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t p = uint32_t(v[i]) * A.lw_fold[i];
        uint32_t f = add_mod(p & 0xFFFFu, p >> 16);
        if (A.low_rate && i == 0) f = add_mod(f, A.lw0);
        v[i] = uint16_t(f);
    }
    __syncthreads();
    RS_ESTAMP(3);
    walsh(v, A.u);
    RS_ESTAMP(4);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t rcv = inl ? (A.received[i >> 5] >> (i & 31)) & 1u : (A.state[i] >> 1) & 1u;
        A.rowinfo[i] = v[i] | (rcv ? 0u : 0x10000u);
    }
    RS_ESTAMP(5);
}

}  // namespace

hipError_t launch_eval_poly(const EvalArgs &A, hipStream_t s) {
    const size_t lds = size_t(2) << A.u;
    static bool attr_set = false;  // benign race: idempotent attribute call
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_eval_poly),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 2 << 16);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const uint32_t threads = A.u >= 13 ? 1024 : (A.u >= 4 ? 1u << (A.u - 3) : 1);
    k_eval_poly<<<1, threads < 64 ? 64 : threads, lds, s>>>(A);
    return hipGetLastError();
}

}  // namespace rs
