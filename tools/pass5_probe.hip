// Config-5 pass timing (development tool, not shipped): the three passes of a
// 32768:32768 x 64 KiB HighRate encode (IFFT level 0, K = 8 from the originals;
// fused IFFT + FFT top level, K = 7; FFT level 0, K = 8 to the recovery rows),
// each timed back to back with HIP events, plus a 2 GiB device copy.
// Build variants with -D flags of rs_kernels.hip (A/B; profiles/r04a/ab_stream_pass.md).
// Run: tools/_probe/pass5_<variant> [rows] [shard bytes] [iters]
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

__global__ void k_copy(const uint4 *in, uint4 *out, size_t n) {
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        out[i] = in[i];
}

template <typename F>
static double time_us(F &&launch, int iters) {
    launch();
    CK(hipDeviceSynchronize());
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
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 32768, S = argc > 2 ? atoi(argv[2]) : 65536;
    const int iters = argc > 3 ? atoi(argv[3]) : 5;
    const auto &T = rs::tables();
    uint32_t *d_tw;
    CK(hipMalloc(&d_tw, T.perm_by_skew.size() * 4));
    CK(hipMemcpy(d_tw, T.perm_by_skew.data(), T.perm_by_skew.size() * 4, hipMemcpyHostToDevice));
    const size_t bytes = size_t(n) * S;
    uint8_t *orig, *W, *rec;
    CK(hipMalloc(&orig, bytes));
    CK(hipMalloc(&W, bytes));
    CK(hipMalloc(&rec, bytes));
    {  // pseudo-random originals (a constant fill would hide errors)
        std::vector<uint8_t> h(bytes);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (size_t i = 0; i < bytes; ++i) x ^= x << 13, x ^= x >> 7, x ^= x << 17, h[i] = uint8_t(x);
        CK(hipMemcpy(orig, h.data(), bytes, hipMemcpyHostToDevice));
    }
    CK(hipMemset(W, 0, bytes));
    uint32_t L = 0;
    while ((1u << L) < n) ++L;
    const uint32_t K0 = 8, K1 = L - K0;
    rs::PassArgs A;
    A.n = n;
    A.packs = S / 8;
    A.tw = d_tw;
    A.work_stride = S;
    rs::PassArgs P = A;  // IFFT level 0 (rows of the originals, skew offset n)
    P.src[0] = rs::RowMap{orig, S, 0, n};
    P.nsrc = 1;
    P.work_out = W;
    P.ifft_delta = n;
    P.nsets = n >> K0;
    P.a = 0;
    rs::PassArgs Q = A;  // fused top level: IFFT (offset n) + FFT (offset 0)
    Q.work_in = W;
    Q.work_out = W;
    Q.ifft_delta = n;
    Q.nsets = n >> K1;
    Q.a = K0;
    rs::PassArgs F = A;  // FFT level 0 into the recovery rows
    F.work_in = W;
    F.dst = rs::RowMap{rec, S, 0, n};
    F.nsets = n >> K0;
    F.a = 0;
    const double gb = 2.0 * double(bytes) / 1e9;
    const size_t n16 = bytes / 16;
    const double tc = time_us([&] { k_copy<<<8192, 256>>>((const uint4 *)orig, (uint4 *)rec, n16); }, iters);
    printf("copy 2x%zu B  %9.1f us  %6.2f TB/s\n", bytes, tc, gb / tc * 1e3);
    auto run = [&](const char *name, int K, int flags, const rs::PassArgs &X) {
        const double t = time_us([&] { CK(rs::launch_pass(K, flags, X, 0)); }, iters);
        printf("%-10s K=%d  %9.1f us  %6.2f TB/s  (%s)\n", name, K, t, gb / t * 1e3, rs::launch_name_buf());
        return t;
    };
    const double t1 = run("ifft", K0, rs::kIfft, P);
    const double t2 = run("ifft+fft", K1, rs::kIfft | rs::kFft, Q);
    const double t3 = run("fft", K0, rs::kFft, F);
    printf("encode (3 passes) %9.1f us  %7.1f GiB/s\n", t1 + t2 + t3, 2.0 * bytes / (t1 + t2 + t3) * 1e6 / (1u << 30));
    {  // FNV-1a of the recovery rows: compare across -D variants of rs_kernels.hip
        CK(hipMemset(W, 0, bytes));
        CK(rs::launch_pass(K0, rs::kIfft, P, 0));
        CK(rs::launch_pass(K1, rs::kIfft | rs::kFft, Q, 0));
        CK(rs::launch_pass(K0, rs::kFft, F, 0));
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> b(bytes);
        CK(hipMemcpy(b.data(), rec, bytes, hipMemcpyDeviceToHost));
        uint64_t h = 0xcbf29ce484222325ull;
        for (uint8_t v : b) h = (h ^ v) * 0x100000001b3ull;
        printf("recovery hash %016llx\n", (unsigned long long)h);
    }
    return 0;
}
