// Development probe: largest kernel-argument struct HIP accepts on this stack,
// and the back-to-back launch time as the argument grows.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int W>
struct Big {
    unsigned v[W];
};
template <int W>
__global__ void k_big(const Big<W> a, unsigned *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = a.v[W - 1] + a.v[blockIdx.x % W];
}
template <int W>
void run(unsigned *d) {
    Big<W> a{};
    for (int i = 0; i < W; ++i) a.v[i] = i;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i) k_big<W><<<256, 64>>>(a, d);
    hipEventRecord(e0);
    for (int i = 0; i < 1000; ++i) k_big<W><<<256, 64>>>(a, d);
    hipEventRecord(e1);
    hipError_t err = hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned h = 0;
    hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("kernarg %6d B: %s, out %u (want %u), %.2f us/launch\n", int(sizeof(a)), hipGetErrorString(err), h,
           unsigned(W - 1), ms);
}
int main() {
    unsigned *d;
    hipMalloc(&d, 4096);
    run<16>(d);
    run<512>(d);
    run<1024>(d);
    run<1536>(d);
    run<2048>(d);
    run<4096>(d);
    return 0;
}
