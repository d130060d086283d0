// Lane-kernel timing (development tool): k_lane<L> (rs_lane.hip) encodes of an
// n:n x S stripe, back-to-back launch time and per-workgroup s_memrealtime
// stamps (wave 0 and the last wave; the instruction stream's arrival, not memory).
// Build: bash tools/build_lane_probe.sh <name> [flags]   Run: tools/_probe/<name> [n] [S]
#ifndef RS_LANE_NO_STAMPS
#define RS_LANE_STAMPS 1
#endif
#include "../reed-solomon-simd_amd/csrc/rs_lane.hip"

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
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1024, S = argc > 2 ? atoi(argv[2]) : 1024;
    uint32_t L = 0;
    while ((1u << L) < n) ++L;
    const auto &T = rs::tables();
    // RS_LANE_BASIS: 8-word basis images (rs_codec.cpp basis_images), else the 16-word tables
    const int tw = RS_LANE_BASIS ? 8 : rs::kPerm2Words;
    const uint32_t nimg = 65536u / n;
    const size_t words = size_t(n - 1) * tw;
    std::vector<uint32_t> h(words * nimg);
    for (uint32_t t = 0; t < nimg; ++t)
        for (uint32_t b = 0; b < L; ++b)
            for (uint32_t g = 0; g < (n >> (b + 1)); ++g) {
                const uint32_t slot = n - (n >> b) + g, idx = (g << (b + 1)) + (1u << b) + t * n - 1;
                uint32_t *dst = &h[t * words + size_t(slot) * tw];
                if (RS_LANE_BASIS) {
                    const uint16_t lm = T.skew[idx];
                    auto P = [&](int i) -> uint32_t { return lm == 65535 ? 0u : T.mul(uint16_t(1u << i), lm); };
                    for (int f = 0; f < 4; ++f) {
                        dst[2 * f] = P(2 * f) | (P(2 * f + 1) << 16);
                        dst[2 * f + 1] = P(8 + 2 * f) | (P(9 + 2 * f) << 16);
                    }
                } else {
                    std::copy_n(&T.perm2_by_skew[size_t(idx) * tw], tw, dst);
                }
            }
    uint32_t *d_img;
    CK(hipMalloc(&d_img, h.size() * 4));
    CK(hipMemcpy(d_img, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    uint8_t *orig, *rec;
    CK(hipMalloc(&orig, size_t(n) * S));
    CK(hipMalloc(&rec, size_t(n) * S));
    {
        std::vector<uint8_t> hin(size_t(n) * S);
        uint32_t x = 12345;
        for (auto &c : hin) c = uint8_t((x = x * 1103515245u + 12345u) >> 16);
        CK(hipMemcpy(orig, hin.data(), hin.size(), hipMemcpyHostToDevice));
    }
    rs::MonoArgs A;
    A.elems = 2;
    A.packs = S / 4;
    A.packs_per_xcd = (A.packs + 7) / 8;
    A.src[0] = rs::RowMap{orig, S, 0, n};
    A.nsrc = 1;
    A.dst = rs::RowMap{rec, S, 0, n};
    A.chunks = 1;
    A.img = d_img;
    A.img_words = words;
    A.ifft_img = 1;
    A.fft_img = 0;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int i = 0; i < 20; ++i) CK(rs::launch_lane(int(L), A, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 400;
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) CK(rs::launch_lane(int(L), A, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint32_t> out(size_t(n) * S / 4);
    CK(hipMemcpy(out.data(), rec, out.size() * 4, hipMemcpyDeviceToHost));
    uint64_t hsh = 1469598103934665603ull;
    for (uint32_t w : out) hsh = (hsh ^ w) * 1099511628211ull;
    printf("k_lane<%u> (basis %d) %u:%u x %u: %.3f us per launch back to back, output hash %016llx\n", L, RS_LANE_BASIS, n, n,
           S, ms * 1e3f / reps, (unsigned long long)hsh);
#ifdef RS_LANE_STAMPS
    CK(rs::launch_lane(int(L), A, s));
    CK(hipStreamSynchronize(s));
    std::vector<uint64_t> st(4096 * 2 * 12);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(rs::g_lane_stamps), st.size() * 8));
    const uint32_t grid = 8u * A.packs_per_xcd;
    const char *names[10] = {"entry", "loads issued", "A1 written", "column ready", "IFFT phase A",
                             "remap 1", "phase B", "remap 2", "FFT phase A", "stores issued"};
    for (int w = 0; w < 2; ++w) {
        printf("%s:\n", w ? "last wave" : "wave 0");
        for (int i = 1; i < 10; ++i) {
            std::vector<double> d;
            for (uint32_t b = 0; b < grid; ++b) d.push_back(double(st[(b * 2 + w) * 12 + i] - st[(b * 2 + 0) * 12 + 0]) / 100.0);
            std::sort(d.begin(), d.end());
            printf("  %-14s median %6.2f us  (min %6.2f max %6.2f)\n", names[i], d[d.size() / 2], d[0], d.back());
        }
    }
#endif
    return 0;
}
