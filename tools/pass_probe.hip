// Latency probe for the pass kernels (development tool, not shipped).
//
// Times back-to-back launches of single pass kernels at the headline geometry
// (1024 rows x 1024-byte shards) plus an empty kernel and a plain copy, so the
// fixed cost of a pass (launch, loads, staging, barriers, store) can be told
// apart from its butterfly layers.  Built three ways by tools/Makefile: full,
// -DRS_PROBE_SKIP_XFORM and -DRS_PROBE_SKIP_STAGE.
#include "../reed-solomon-simd_amd/csrc/rs_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../reed-solomon-simd_amd/csrc/gf_tables.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_empty() {}
__global__ void k_copy(const uint4 *in, uint4 *out, size_t n) {
    size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

template <typename F>
static double time_us(F &&launch, int iters) {
    for (int i = 0; i < 20; ++i) launch();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.0 / iters;
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1024, S = argc > 2 ? atoi(argv[2]) : 1024;
    const int iters = 2000;
    const auto &T = rs::tables();
    uint32_t *d_tw, *d_lut;
    CK(hipMalloc(&d_tw, T.perm_by_skew.size() * 4));
    CK(hipMalloc(&d_lut, T.perm_by_log.size() * 4));
    CK(hipMemcpy(d_tw, T.perm_by_skew.data(), T.perm_by_skew.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lut, T.perm_by_log.data(), T.perm_by_log.size() * 4, hipMemcpyHostToDevice));
    const size_t bytes = size_t(n) * S;
    uint8_t *orig, *W, *rec;
    CK(hipMalloc(&orig, bytes));
    CK(hipMalloc(&W, bytes));
    CK(hipMalloc(&rec, bytes));
    std::vector<uint8_t> h(bytes);
    for (size_t i = 0; i < bytes; ++i) h[i] = uint8_t(i * 2654435761u >> 13);
    CK(hipMemcpy(orig, h.data(), bytes, hipMemcpyHostToDevice));

    printf("n=%u S=%u\n", n, S);
    printf("empty<<<256,64>>>          %7.2f us\n", time_us([&] { k_empty<<<256, 64>>>(); }, iters));
    const size_t n16 = bytes / 16;
    printf("copy %zu B                 %7.2f us\n", bytes,
           time_us([&] { k_copy<<<(n16 + 255) / 256, 256>>>((const uint4 *)orig, (uint4 *)W, n16); }, iters));

    uint32_t L = 0;
    while ((1u << L) < n) ++L;
    const uint32_t K0 = L / 2, K1 = L - K0;
    rs::PassArgs A;
    A.n = n;
    A.packs = S / 8;
    A.slices = (A.packs + 63) / 64;
    A.tw = d_tw;
    A.lut = d_lut;
    A.work_stride = S;
    // shape sweep at K = 5 (headline split 5 + 5)
    auto sweep = [&](auto lr_c, auto spl_c) {
        constexpr int LRv = decltype(lr_c)::value, SPLv = decltype(spl_c)::value;
        rs::PassArgs P = A;
        P.src[0] = rs::RowMap{orig, S, 0, n};
        P.nsrc = 1;
        P.work_out = W;
        P.ifft_delta = n;
        P.nsets = n >> 5;
        P.a = 0;
        rs::PassArgs Q = A;
        Q.work_in = W;
        Q.work_out = W;
        Q.ifft_delta = n;
        Q.nsets = n >> 5;
        Q.a = 5;
        rs::PassArgs F = A;
        F.work_in = W;
        F.dst = rs::RowMap{rec, S, 0, n};
        F.nsets = n >> 5;
        F.a = 0;
        auto l1 = [&] { CK((rs::launch_k<5, LRv, SPLv>(rs::kIfft, P, 0))); };
        auto l2 = [&] { CK((rs::launch_k<5, LRv, SPLv>(rs::kIfft | rs::kFft, Q, 0))); };
        auto l3 = [&] { CK((rs::launch_k<5, LRv, SPLv>(rs::kFft, F, 0))); };
        printf("K=5 LR=%d SP=%3d  ifft %6.2f  ifft+fft %6.2f  fft %6.2f  encode %6.2f us\n", LRv, 1 << SPLv,
               time_us(l1, iters), time_us(l2, iters), time_us(l3, iters),
               time_us([&] { l1(); l2(); l3(); }, iters));
    };
    if (n == 1024) {
        using std::integral_constant;
        sweep(integral_constant<int, 3>{}, integral_constant<int, 6>{});
        sweep(integral_constant<int, 3>{}, integral_constant<int, 4>{});
        sweep(integral_constant<int, 3>{}, integral_constant<int, 5>{});
        sweep(integral_constant<int, 2>{}, integral_constant<int, 3>{});
        sweep(integral_constant<int, 2>{}, integral_constant<int, 4>{});
        sweep(integral_constant<int, 2>{}, integral_constant<int, 5>{});
        sweep(integral_constant<int, 1>{}, integral_constant<int, 2>{});
        sweep(integral_constant<int, 1>{}, integral_constant<int, 3>{});
        sweep(integral_constant<int, 1>{}, integral_constant<int, 4>{});
    }
    return 0;
}
