// Sync-cost probe (development tool): kernel boundary vs in-kernel barriers
// among the workgroups of one column slice, vs a hipGraph of three launches.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_empty() {}

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Barrier among the `members` workgroups sharing counter `ctr` (monotonic).
__device__ void group_barrier(uint32_t *ctr, uint32_t target, uint32_t *fail) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t spins = 0;
        while (int32_t(ld_sc1(ctr) - target) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) {
                *fail = 1;
                break;
            }
        }
    }
    __syncthreads();
}

// grid = groups * members; group of block b = b % groups (XCD-affine when groups == 8)
__global__ void k_barriers(uint32_t *ctrs, uint32_t groups, uint32_t members, uint32_t seq, int nbar, uint32_t *data,
                           int words, uint32_t *fail) {
    const uint32_t grp = blockIdx.x % groups, mem = blockIdx.x / groups;
    uint32_t *ctr = ctrs + grp * 32;
    uint32_t acc = 0;
    for (int b = 0; b < nbar; ++b) {
        for (int w = threadIdx.x; w < words; w += blockDim.x) st_sc1(data + (size_t(blockIdx.x) * words + w), acc + w);
        group_barrier(ctr, (seq * nbar + b + 1) * members, fail);
        const uint32_t src = (grp + ((mem + 1) % members) * groups);
        for (int w = threadIdx.x; w < words; w += blockDim.x) acc += ld_sc1(data + (size_t(src) * words + w));
    }
    if (acc == 0xdeadbeef) *fail = 2;
}

int main() {
    const int iters = 2000;
    uint32_t *ctrs, *data, *fail;
    CK(hipMalloc(&ctrs, 4096));
    CK(hipMemset(ctrs, 0, 4096));
    CK(hipMalloc(&data, 64 << 20));
    CK(hipMalloc(&fail, 4));
    CK(hipMemset(fail, 0, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char *name, auto &&f) {
        for (int i = 0; i < 10; ++i) f(i);
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < iters; ++i) f(10 + i);
        CK(hipEventRecord(b, 0));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-48s GPU %7.2f us   host enqueue %6.2f us\n", name, ms * 1000 / iters,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
    };
    run("empty x1", [&](int) { k_empty<<<256, 256>>>(); });
    run("empty x3", [&](int) {
        k_empty<<<256, 256>>>();
        k_empty<<<256, 256>>>();
        k_empty<<<256, 256>>>();
    });
    uint32_t seq = 0;
    for (int words : {0, 1024}) {
        for (int g : {8, 1}) {
            for (int nbar : {1, 2}) {
                CK(hipMemset(ctrs, 0, 4096));
                seq = 0;
                char name[96];
                snprintf(name, sizeof name, "256 WGs, %d groups, %d barriers, %d words/WG", g, nbar, words);
                run(name, [&](int) {
                    k_barriers<<<256, 256>>>(ctrs, g, 256 / g, seq++, nbar, data, words, fail);
                });
            }
        }
    }
    // hipGraph of three empty kernels
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    k_empty<<<256, 256, 0, s>>>();
    k_empty<<<256, 256, 0, s>>>();
    k_empty<<<256, 256, 0, s>>>();
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    CK(hipEventRecord(a, s));
    for (int i = 0; i < iters; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    auto t1 = std::chrono::steady_clock::now();
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-48s GPU %7.2f us   host enqueue %6.2f us\n", "graph of 3 empty", ms * 1000 / iters,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
    uint32_t f = 0;
    CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
    printf("fail flag %u\n", f);
    return 0;
}
