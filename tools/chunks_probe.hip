// Multi-chunk column kernel timing (development tool): k_chunks (rs_chunks.hip)
// on one shape, back-to-back launch time and per-workgroup s_memrealtime stamps
// of wave 0 and the last wave (RS_CHUNK_STAMPS).
// Build: bash tools/build_chunks_probe.sh   Run: tools/_probe/chunks_probe N M S high|low [e2|e4]
#ifndef RS_CHUNK_NO_STAMPS
#define RS_CHUNK_STAMPS 1
#endif
#include "../reed-solomon-simd_amd/csrc/rs_chunks.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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
    if (argc < 5) {
        fprintf(stderr, "usage: chunks_probe N M S high|low [e2|e4]\n");
        return 2;
    }
    const uint32_t N = atoi(argv[1]), M = atoi(argv[2]), S = atoi(argv[3]);
    const bool high = std::string(argv[4]) == "high";
    const bool e2 = argc > 5 ? std::string(argv[5]) == "e2" : S <= 1024;
    auto p2 = [](uint32_t x) { uint32_t n = 1; while (n < x) n <<= 1; return n; };
    const uint32_t n = high ? p2(M) : p2(N);
    uint32_t L = 0;
    while ((1u << L) < n) ++L;
    const uint32_t C = high ? (N + n - 1) / n : (M + n - 1) / n;
    const auto &T = rs::tables();
    const int tw = e2 ? rs::kPerm2Words : rs::kPermWords;
    const std::vector<uint32_t> &skew_tabs = e2 ? T.perm2_by_skew : T.perm_by_skew;
    const uint32_t nimg = 65536u / n;
    const size_t words = size_t(n - 1) * 8;
    std::vector<uint32_t> h(words * nimg);
    // 4-element packs: the 20-word tables; 2-element: 8-word basis images (rs_chunks.hip CTabsBasis)
    for (uint32_t t = 0; t < nimg; ++t)
        for (uint32_t b = 0; b < L; ++b)
            for (uint32_t g = 0; g < (n >> (b + 1)); ++g) {
                const uint32_t slot = n - (n >> b) + g, idx = (g << (b + 1)) + (1u << b) + t * n - 1;
                const uint16_t lm = T.skew[idx];
                uint32_t *dst = &h[t * words + size_t(slot) * 8];
                auto P = [&](int i) -> uint32_t { return lm == 65535 ? 0u : T.mul(uint16_t(1u << i), lm); };
                if (e2) {
                    for (int f = 0; f < 4; ++f) {
                        dst[2 * f] = P(2 * f) | (P(2 * f + 1) << 16);
                        dst[2 * f + 1] = P(8 + 2 * f) | (P(9 + 2 * f) << 16);
                    }
                } else {
                    for (int B = 0; B < 2; ++B) {
                        const int j = 8 * B;
                        dst[4 * B] = P(j) | (P(j + 1) << 16);
                        dst[4 * B + 1] = P(j + 3) | (P(j + 4) << 16);
                        dst[4 * B + 2] = P(j + 6) | (P(j + 7) << 16);
                        dst[4 * B + 3] = P(j + 2) | (P(j + 5) << 16);
                    }
                }
            }
    uint32_t *d_img;
    CK(hipMalloc(&d_img, h.size() * 4));
    CK(hipMemcpy(d_img, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    uint8_t *orig, *rec;
    CK(hipMalloc(&orig, size_t(N) * S));
    CK(hipMalloc(&rec, size_t(M) * S));
    {
        std::vector<uint8_t> hin(size_t(N) * S);
        uint32_t x = 12345;
        for (auto &c : hin) c = uint8_t((x = x * 1103515245u + 12345u) >> 16);
        CK(hipMemcpy(orig, hin.data(), hin.size(), hipMemcpyHostToDevice));
    }
    rs::MonoCore A;
    A.elems = e2 ? 2 : 4;
    A.packs = e2 ? S / 4 : S / 8;
    A.packs_per_xcd = (A.packs + 7) / 8;
    A.src[0] = rs::RowMap{orig, S, 0, N};
    A.nsrc = 1;
    A.dst = rs::RowMap{rec, S, 0, M};
    A.chunks = C;
    A.img = d_img;
    A.img_words = words;
    A.ifft_img = high ? 1 : 0;
    A.ifft_img_step = high ? 1 : 0;
    A.fft_img = high ? 0 : 1;
    A.fft_img_step = high ? 0 : 1;
    const int iters = 1000;
    const int pw = getenv("PW") ? atoi(getenv("PW")) : 1;
    auto go = [&] { CK(rs::launch_chunks(int(L), high, A, 0, pw)); };
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
    std::vector<uint32_t> out(size_t(M) * S / 4);
    CK(hipMemcpy(out.data(), rec, out.size() * 4, hipMemcpyDeviceToHost));
    uint64_t hsh = 1469598103934665603ull;
    for (uint32_t w : out) hsh = (hsh ^ w) * 1099511628211ull;
    printf("k_chunks<%u, %d, %s, %d> %u:%u x %u B, %u chunks: %.2f us/launch (back-to-back), output hash %016llx\n", L,
           e2 ? 2 : 4, high ? "high" : "low", pw, N, M, S, C, ms * 1000 / iters, (unsigned long long)hsh);
#ifdef RS_CHUNK_STAMPS
    CK(hipDeviceSynchronize());
    go();
    CK(hipDeviceSynchronize());
    const uint32_t wgs = 8 * (((A.packs + pw - 1) / pw + 7) / 8);
    std::vector<uint64_t> st(4096 * 2 * 8);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(rs::g_chunk_stamps), st.size() * 8));
    const char *names[8] = {"entry", "tables written", "transform 1", "loop done", "barrier", "fft done", "stored", ""};
    for (int w = 0; w < 2; ++w)
        for (int i = 0; i < 7; ++i) {
            std::vector<double> v;
            for (uint32_t g = 0; g < wgs; ++g) {
                const uint64_t t0 = st[(g * 2 + 0) * 8 + 0], t = st[(g * 2 + w) * 8 + i];
                if (t && t0) v.push_back((double(t) - double(t0)) * 0.01);
            }
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            printf("%s %-15s min %6.2f  med %6.2f  max %6.2f us\n", w ? "last wave" : "wave 0   ", names[i], v.front(),
                   v[v.size() / 2], v.back());
        }
#endif
    return 0;
}
