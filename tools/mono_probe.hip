// Column-kernel timing (development tool): headline encode (1024:1024 x 1 KiB,
// high rate) through k_mono, back-to-back launch time and per-workgroup
// s_memrealtime stamps (each stamp first waits for the wave's memory ops).
// Build: make -C tools _build/mono_probe   Run: tools/_build/mono_probe [n] [S]
#ifndef RS_MONO_NO_STAMPS
#define RS_MONO_STAMPS 1
#endif
#ifdef RS_MONO_SRC  // A/B: another version of the kernel source (include path: csrc)
#include RS_MONO_SRC
#else
#include "../reed-solomon-simd_amd/csrc/rs_mono.hip"
#endif

#include <algorithm>
#include <string>
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

__global__ void k_empty_lds(int x) {
    extern __shared__ uint32_t lds_[];
    if (x) lds_[threadIdx.x] = x;
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 1024, S = argc > 2 ? atoi(argv[2]) : 1024;
    uint32_t L = 0;
    while ((1u << L) < n) ++L;
    const auto &T = rs::tables();
    // "...2" in the mode argument: 2-element packs (the codec's decode format)
    const bool e2 = argc > 3 && std::string(argv[3]).find('2') != std::string::npos;
    const int tw = e2 ? rs::kPerm2Words : rs::kPermWords;
    const std::vector<uint32_t> &skew_tabs = e2 ? T.perm2_by_skew : T.perm_by_skew;
    const uint32_t nimg = 65536u / n;
    // 2-element packs built with RS_MONO_BASIS: 8-word basis images (rs_mono.hip Stage::kBasis)
    const bool basis = e2 && RS_MONO_BASIS;
    const size_t tabw = basis ? 8 : size_t(tw);
    const size_t words = size_t(n - 1) * tabw;
    std::vector<uint32_t> h(words * nimg);
    for (uint32_t t = 0; t < nimg; ++t)
        for (uint32_t b = 0; b < L; ++b)
            for (uint32_t g = 0; g < (n >> (b + 1)); ++g) {
                const uint32_t slot = n - (n >> b) + g, idx = (g << (b + 1)) + (1u << b) + t * n - 1;
                if (!basis) {
                    std::copy_n(&skew_tabs[size_t(idx) * tw], tw, &h[t * words + size_t(slot) * tw]);
                    continue;
                }
                const uint16_t lm = T.skew[idx];
                auto P = [&](int i) -> uint32_t { return lm == 65535 ? 0u : T.mul(uint16_t(1u << i), lm); };
                uint32_t *dst = &h[t * words + size_t(slot) * 8];
                for (int f = 0; f < 4; ++f) {
                    dst[2 * f] = P(2 * f) | (P(2 * f + 1) << 16);
                    dst[2 * f + 1] = P(8 + 2 * f) | (P(9 + 2 * f) << 16);
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
    CK(hipMemset(rec, 0, size_t(n) * S));
    rs::MonoArgs A;
    A.elems = e2 ? 2 : 4;
    A.packs = e2 ? S / 4 : S / 8;
    A.packs_per_xcd = (A.packs + 7) / 8;
    A.src[0] = rs::RowMap{orig, S, 0, n};
    A.nsrc = 1;
    A.dst = rs::RowMap{rec, S, 0, n};
    A.chunks = 1;
    A.img = d_img;
    A.img_words = words;
    A.ifft_img = 1;
    A.fft_img = 0;
    // decode mode: 2^L work rows = n/2 recovery + n/2 originals (high rate),
    // recovery all present, originals all missing (the 100 % loss pattern)
    const bool dec = argc > 3 && argv[3][0] == 'd';
    int mode = rs::kMonoEncodeHigh;
    std::vector<uint32_t> lwf(n, 1);
    uint16_t *d_lw = nullptr;
    uint32_t *d_lut = nullptr;
    if (dec) {
        mode = rs::kMonoDecode;
        A.src[0] = rs::RowMap{orig, S, 0, n / 2};
        A.src[1] = rs::RowMap{orig, S, n / 2, n};
        A.nsrc = 2;
        A.dst = rs::RowMap{rec, S, n / 2, n};
        A.ifft_img = 0;
        A.fused_eval = 1;
        A.end = n;
        std::vector<uint16_t> lw(T.lw_fold.begin() + (n - 1), T.lw_fold.begin() + (2 * n - 1));
        CK(hipMalloc(&d_lw, n * 2));
        CK(hipMemcpy(d_lw, lw.data(), n * 2, hipMemcpyHostToDevice));
        A.lw_fold = d_lw;
        const std::vector<uint32_t> &lut = e2 ? T.perm2_by_log : T.perm_by_log;
        CK(hipMalloc(&d_lut, lut.size() * 4));
        CK(hipMemcpy(d_lut, lut.data(), lut.size() * 4, hipMemcpyHostToDevice));
        A.lut = d_lut;
        // "d1": the 1 % pattern (recovery 0..11 and originals 0..n/2-12 received)
        const bool one = argv[3][1] == '1';
        // "...s": the split plan (restored rows = the upper half's erased originals)
        if (std::string(argv[3]).find('s') != std::string::npos) A.split = 1, A.out_half = 1;
        // "...n": the destination narrowed to the erased rows' span, as rs_codec.cpp
        // decode_dev passes it since r06 (1 %: the last 11 rows)
        if (one && std::string(argv[3]).find('n') != std::string::npos)
            A.dst = rs::RowMap{rec + size_t(n / 2 - 11) * S, S, n - 11, n};
        for (uint32_t r = 0; r < n; ++r) {
            const bool rcv = one ? (r < 12 || (r >= n / 2 && r < n - 11)) : r < n / 2;
            if (rcv) A.received[r >> 5] |= 1u << (r & 31);
            else A.erased[r >> 5] |= 1u << (r & 31);
        }
    }
    // "hi" / "hf" (n = 2048): the half-split kernels of a 4096:4096 HighRate encode,
    // kMonoHalfIEnc (IFFT halves into the work rows) / kMonoHalfFEnc (top layer + FFT halves)
    uint32_t halves = 0;
    if (argc > 3 && argv[3][0] == 'h') {
        uint8_t *o2, *w2, *r2;
        CK(hipMalloc(&o2, size_t(2 * n) * S));
        CK(hipMalloc(&w2, size_t(2 * n) * S));
        CK(hipMalloc(&r2, size_t(2 * n) * S));
        CK(hipMemset(o2, 0x37, size_t(2 * n) * S));
        CK(hipMemset(w2, 0x21, size_t(2 * n) * S));
        std::vector<uint32_t> top(2 * tw);
        for (int k = 0; k < 2; ++k)  // skew index 2047 + delta: delta 4096 (IFFT), 0 (FFT)
            std::copy_n(&skew_tabs[size_t(2047 + (k == 0 ? 4096 : 0)) * tw], tw, &top[k * tw]);
        uint32_t *d_top;
        CK(hipMalloc(&d_top, top.size() * 4));
        CK(hipMemcpy(d_top, top.data(), top.size() * 4, hipMemcpyHostToDevice));
        A.top_i = d_top;
        A.top_f = d_top + tw;
        halves = 2;
        if (argv[3][1] == 'i') {
            mode = rs::kMonoHalfIEnc;
            A.src[0] = rs::RowMap{o2, S, 0, 2 * n};
            A.dst = rs::RowMap{w2, S, 0, 2 * n};
            A.ifft_img = 2;
            A.ifft_img_step = 1;
        } else {
            mode = rs::kMonoHalfFEnc;
            A.src[0] = rs::RowMap{w2, S, 0, 2 * n};
            A.dst = rs::RowMap{r2, S, 0, 2 * n};
            A.fft_img = 0;
            A.fft_img_step = 1;
        }
    }
    const int iters = 1000;
    auto go = [&] { CK(halves ? rs::launch_mono_half(mode, halves, A, 0) : rs::launch_mono(mode, int(L), A, 0)); };
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
    uint64_t hsh = 1469598103934665603ull;
    {  // output hash (A/B builds must agree)
        std::vector<uint32_t> out(size_t(n) * S / 4);
        CK(hipMemcpy(out.data(), rec, out.size() * 4, hipMemcpyDeviceToHost));
        for (uint32_t w : out) hsh = (hsh ^ w) * 1099511628211ull;
    }
    printf("mono %s%s%s n=%u S=%u: %.2f us/launch (back-to-back), output hash %016llx\n", dec ? "decode" : "encode",
           A.split ? " split" : "", e2 ? " e2" : "", n, S, ms * 1000 / iters, (unsigned long long)hsh);
    {  // floor: an empty kernel with the same grid, block and LDS
        const size_t lds = size_t(rs::Stage<10, 1>::words_dec) * 4;
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_empty_lds), hipFuncAttributeMaxDynamicSharedMemorySize,
                               int(lds)));
        const uint32_t grid = 8 * A.packs_per_xcd;
        for (int i = 0; i < 20; ++i) k_empty_lds<<<grid, 512, lds, 0>>>(0);
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < iters; ++i) k_empty_lds<<<grid, 512, lds, 0>>>(0);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("empty kernel, same grid/block/LDS: %.2f us/launch (back-to-back)\n", ms * 1000 / iters);
    }
#ifdef RS_MONO_STAMPS
    CK(hipDeviceSynchronize());
    go();
    CK(hipDeviceSynchronize());
    const uint32_t wgs = 8 * A.packs_per_xcd * (halves ? halves : 1);
    std::vector<uint64_t> st(4096 * 24);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(rs::g_mono_stamps), st.size() * 8));
    // s_memrealtime is per XCD: entry spread within each XCD's workgroups
    // (b % 8), stages as per-workgroup deltas from the workgroup's wave-0 entry
    {
        double sp = 0;
        for (uint32_t x = 0; x < 8; ++x) {
            uint64_t lo = ~0ull, hi = 0;
            for (uint32_t w = x; w < wgs; w += 8) lo = std::min(lo, st[w * 24 + 12]), hi = std::max(hi, st[w * 24 + 12]);
            sp = std::max(sp, (hi - lo) * 0.01);
        }
        printf("entry spread within an XCD (worst XCD): %.2f us\n", sp);
    }
    const char *names[24] = {"start", "loaded", "eval done", "ifft A done", "remap1 done", "ifft B done", "split done", "entry",
                             "fft B done", "remap2 done", "fft C done", "stored", "entry wave0", "loads issued",
                             "walsh1 done", "lw landed", "shared issued", "rows issued", "priv issued", "walsh1 in-wave",
                             "walsh2 in-wave", "", "", ""};
    const int order[] = {12, 7, 0, 16, 17, 18, 19, 14, 15, 20, 2, 13, 1, 3, 4, 5, 6, 8, 9, 10, 11};
    for (int i : order) {
        std::vector<double> v;
        for (uint32_t w = 0; w < wgs; ++w) v.push_back((double(st[w * 24 + i]) - double(st[w * 24 + 12])) * 0.01);
        std::sort(v.begin(), v.end());
        printf("%-12s min %6.2f  med %6.2f  max %6.2f us\n", names[i], v.front(), v[v.size() / 2], v.back());
    }
#endif
    return 0;
}
