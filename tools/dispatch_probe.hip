// Workgroup dispatch spread of a column-kernel-shaped grid on an idle GPU
// (development tool): 128 workgroups, entry timestamps per workgroup, for
// several block sizes / LDS sizes / kernel-argument sizes.
// Build: hipcc --offload-arch=gfx950 -O3 dispatch_probe.hip -o _build/dispatch_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__device__ uint64_t g_stamp[4096][2];

struct Big {
    uint32_t w[180];
};

template <typename A>
__global__ void k_stamp(A a, int x) {
    extern __shared__ uint32_t lds_[];
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) g_stamp[blockIdx.x][0] = t;
    if (x) lds_[threadIdx.x] = a.w[threadIdx.x % 4];
    __syncthreads();
    if (threadIdx.x == 0) g_stamp[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
}

struct Small {
    uint32_t w[4];
};

template <typename A>
void run(const char *name, int grid, int block, size_t lds) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_stamp<A>), hipFuncAttributeMaxDynamicSharedMemorySize,
                           160 * 1024));
    A a{};
    std::vector<double> spread, all;
    for (int rep = 0; rep < 20; ++rep) {
        CK(hipDeviceSynchronize());
        k_stamp<A><<<grid, block, lds, 0>>>(a, 0);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> st(4096 * 2);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamp), st.size() * 8));
        // s_memrealtime is per XCD: spreads within each group of blocks b % 8 (one XCD
        // under round-robin placement), the worst of the 8
        double sp = 0, al = 0;
        for (int x = 0; x < 8; ++x) {
            uint64_t t0 = ~0ull, t1 = 0, e1 = 0;
            for (int b = x; b < grid; b += 8) {
                t0 = std::min(t0, st[2 * b]);
                t1 = std::max(t1, st[2 * b]);
                e1 = std::max(e1, st[2 * b + 1]);
            }
            sp = std::max(sp, (t1 - t0) * 0.01);
            al = std::max(al, (e1 - t0) * 0.01);
        }
        spread.push_back(sp);
        all.push_back(al);
    }
    std::sort(spread.begin(), spread.end());
    std::sort(all.begin(), all.end());
    // back-to-back launch rate
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    for (int i = 0; i < 20; ++i) k_stamp<A><<<grid, block, lds, 0>>>(a, 0);
    CK(hipEventRecord(ea, 0));
    for (int i = 0; i < 500; ++i) k_stamp<A><<<grid, block, lds, 0>>>(a, 0);
    CK(hipEventRecord(eb, 0));
    CK(hipEventSynchronize(eb));
    float ms;
    CK(hipEventElapsedTime(&ms, ea, eb));
    printf("%-34s grid %4d block %4d lds %6zu: entry spread med %.2f us, last done med %.2f us, back-to-back %.2f us\n",
           name, grid, block, lds, spread[spread.size() / 2], all[all.size() / 2], ms * 1000 / 500);
}

int main() {
    run<Big>("big kernarg (720 B)", 128, 512, 98 * 1024);
    run<Small>("small kernarg", 128, 512, 98 * 1024);
    run<Small>("small kernarg, no LDS", 128, 512, 0);
    run<Small>("small kernarg, 16 KB LDS", 128, 512, 16 * 1024);
    run<Small>("small kernarg, 256 thr", 128, 256, 98 * 1024);
    run<Small>("small kernarg, 1024 thr", 128, 1024, 98 * 1024);
    run<Small>("small kernarg, 64 thr", 128, 64, 0);
    run<Small>("256 WGs, 512 thr, 98 KB", 256, 512, 98 * 1024);
    run<Small>("256 WGs, 256 thr, 64 KB", 256, 256, 64 * 1024);
    run<Big>("big kernarg, 1024 thr, 120 KB", 128, 1024, 120 * 1024);
    return 0;
}
