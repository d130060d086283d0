// Host launch-cost probe (development tool): enqueue cost vs kernel-argument size.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

struct Big {
    uint32_t w[60];
};
__global__ void k0() {}
__global__ void k1(uint32_t *p) {
    if (p && threadIdx.x == 1024) *p = 0;
}
__global__ void k8(uint32_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t *q, int e, uint32_t *f) {
    if (p && threadIdx.x == 1024) *p = a + b + c + d + e + (q != f);
}
__global__ void kbig(const Big B) {
    if (threadIdx.x == 1024) ((uint32_t *)nullptr)[B.w[0]] = B.w[59];
}

template <typename F>
void run(const char *name, F &&f) {
    const int iters = 2000;
    for (int i = 0; i < 20; ++i) f();
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto t0 = std::chrono::steady_clock::now();
    hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) f();
    hipEventRecord(b, 0);
    auto t1 = std::chrono::steady_clock::now();
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s GPU %6.2f us  host %6.2f us\n", name, ms * 1000 / iters,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
}

__global__ void klds(int x) {
    extern __shared__ uint32_t l[];
    if (x) l[threadIdx.x] = x;
}

int main() {
    uint32_t *p;
    hipMalloc(&p, 4);
    Big B{};
    hipStream_t s;
    hipStreamCreate(&s);
    hipFuncSetAttribute(reinterpret_cast<const void *>(&klds), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    run("k0 <<<256,256>>>", [&] { k0<<<256, 256>>>(); });
    run("kbig 240B struct", [&] { kbig<<<256, 256>>>(B); });
    run("k0 x3", [&] { k0<<<256, 256>>>(); k0<<<256, 256>>>(); k0<<<256, 256>>>(); });
    run("k1 null stream", [&] { k1<<<256, 256>>>(p); });
    run("k1 stream s", [&] { k1<<<256, 256, 0, s>>>(p); });
    run("k8 stream s", [&] { k8<<<256, 256, 0, s>>>(p, 1, 2, 3, 4, p, 5, p); });
    run("kbig stream s", [&] { kbig<<<256, 256, 0, s>>>(B); });
    run("klds 128x512 100K stream s", [&] { klds<<<128, 512, 100352, s>>>(0); });
    if (getenv("LP_SHORT")) return 0;
    const int grids[] = {8, 128, 256};
    const int blocks[] = {64, 256, 512, 1024};
    const int ldss[] = {0, 16384, 65536, 100352, 163840};
    for (int g : grids)
        for (int b : blocks)
            for (int l : ldss) {
                char name[64];
                snprintf(name, sizeof name, "klds grid %d block %d lds %d", g, b, l);
                run(name, [&] { klds<<<g, b, l, s>>>(0); });
            }
    return 0;
}
