// Chain-kernel phase timing (development tool): headline encode (1024 x 1 KiB
// high rate) as one chain launch, with per-workgroup s_memrealtime stamps.
#define RS_CHAIN_STAMPS 1
#include "../reed-solomon-simd_amd/csrc/rs_kernels.hip"

#include <algorithm>
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

int main(int argc, char **argv) {
    const uint32_t n = 1024, S = 1024;
    const int spl = argc > 1 ? atoi(argv[1]) : 4;
    const auto &T = rs::tables();
    uint32_t *d_tw, *d_lut, *sync, *fault;
    CK(hipMalloc(&d_tw, T.perm_by_skew.size() * 4));
    CK(hipMalloc(&d_lut, T.perm_by_log.size() * 4));
    CK(hipMemcpy(d_tw, T.perm_by_skew.data(), T.perm_by_skew.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lut, T.perm_by_log.data(), T.perm_by_log.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&sync, 1024 * 128));
    CK(hipMemset(sync, 0, 1024 * 128));
    CK(hipMalloc(&fault, 4));
    CK(hipMemset(fault, 0, 4));
    uint8_t *orig, *W, *rec;
    CK(hipMalloc(&orig, n * S));
    CK(hipMalloc(&W, n * S));
    CK(hipMalloc(&rec, n * S));
    CK(hipMemset(orig, 0x37, n * S));
    rs::PassArgs A;
    A.n = n;
    A.packs = S / 8;
    A.tw = d_tw;
    A.lut = d_lut;
    A.work_stride = S;
    A.ifft_delta = n;
    A.ifft_delta_step = n;
    rs::ChainArgs C;
    for (int k = 0; k < 3; ++k) C.ph[k] = A;
    C.ph[0].src[0] = rs::RowMap{orig, S, 0, n};
    C.ph[0].nsrc = 1;
    C.ph[0].work_out = W;
    C.ph[1].work_in = W;
    C.ph[1].work_out = W;
    C.ph[2].work_in = W;
    C.ph[2].dst = rs::RowMap{rec, S, 0, n};
    const uint32_t slices = (A.packs + (1u << spl) - 1) >> spl;
    for (int k = 0; k < 3; ++k) {
        C.ph[k].slices = slices;
        C.ph[k].nsets = 32;
        C.ph[k].a = k == 1 ? 5 : 0;
        C.items[k] = 32;
    }
    C.members = 32;
    C.sync = sync;
    C.fault = fault;
    const int iters = 1000;
    auto go = [&] { CK(rs::launch_chain(rs::kChainEncodeHigh, 5, 5, spl, C, 0)); };
    for (int i = 0; i < 20; ++i) go();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; ++i) go();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("chain encode 1024x1KiB spl=%d: %.2f us/launch (back-to-back)\n", spl, ms * 1000 / iters);
    // one isolated launch for the stamps
    CK(hipDeviceSynchronize());
    go();
    CK(hipDeviceSynchronize());
    const uint32_t wgs = slices * 32;
    std::vector<uint64_t> st(4096 * 32);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(rs::g_chain_stamps), st.size() * 8));
    uint64_t t0 = ~0ull;
    for (uint32_t w = 0; w < wgs; ++w) t0 = std::min(t0, st[w * 32]);
    const char *names[32] = {"start", "phase0 done", "barrier1 out", "phase1 done", "barrier2 out", "phase2 done",
                             "stores drained", "", "p0 staged", "p0 xformed", "p1 staged", "p1 xformed",
                             "p2 staged", "p2 xformed"};
    const int order[] = {0, 8, 9, 1, 2, 10, 11, 3, 4, 12, 13, 5, 6};
    for (int i : order) {
        std::vector<double> v;
        for (uint32_t w = 0; w < wgs; ++w) v.push_back((st[w * 32 + i] - t0) * 0.01);  // 100 MHz -> us
        std::sort(v.begin(), v.end());
        printf("%-14s min %6.2f  med %6.2f  max %6.2f us\n", names[i], v.front(), v[v.size() / 2], v.back());
    }
    uint32_t f = 0;
    CK(hipMemcpy(&f, fault, 4, hipMemcpyDeviceToHost));
    printf("fault %u\n", f);
    return 0;
}
