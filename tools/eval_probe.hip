// eval_poly kernel timing (development tool): stamps inside one launch, and
// back-to-back launch time, at 2^u rows.   tools/_build/eval_probe [u]
#define RS_EVAL_STAMPS 1
#include "../reed-solomon-simd_amd/csrc/rs_eval.hip"

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

int main(int argc, char **argv) {
    const uint32_t u = argc > 1 ? atoi(argv[1]) : 11, n = 1u << u;
    uint16_t *lw;
    uint32_t *ri;
    CK(hipMalloc(&lw, n * 2));
    CK(hipMemset(lw, 1, n * 2));
    CK(hipMalloc(&ri, n * 4));
    rs::EvalArgs E;
    E.u = u;
    E.end = n;
    E.lw_fold = lw;
    E.rowinfo = ri;
    for (uint32_t r = 0; r < n && r < rs::kEvalInlineRows; r += 3) E.erased[r >> 5] |= 1u << (r & 31);
    if (n > rs::kEvalInlineRows) {  // past the inline bitmaps: per-row state bytes (bit 0 erased, bit 1 received)
        std::vector<uint8_t> h(n);
        for (uint32_t r = 0; r < n; ++r) h[r] = r % 3 == 0 ? 1 : 2;
        uint8_t *st;
        CK(hipMalloc(&st, n));
        CK(hipMemcpy(st, h.data(), n, hipMemcpyHostToDevice));
        E.state = st;
    }
    for (int i = 0; i < 10; ++i) CK(rs::launch_eval_poly(E, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < 200; ++i) CK(rs::launch_eval_poly(E, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("eval_poly u=%u: %.2f us/launch back-to-back\n", u, ms * 1000 / 200);
    {  // FNV-1a of the row info: compare across -D variants
        std::vector<uint32_t> out(n);
        CK(hipMemcpy(out.data(), ri, n * 4, hipMemcpyDeviceToHost));
        uint64_t hsh = 0xcbf29ce484222325ull;
        for (uint32_t v : out) hsh = (hsh ^ v) * 0x100000001b3ull;
        printf("rowinfo hash %016llx\n", (unsigned long long)hsh);
    }
    CK(hipDeviceSynchronize());
    CK(rs::launch_eval_poly(E, 0));
    CK(hipDeviceSynchronize());
    uint64_t st[8];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(rs::g_eval_stamps), sizeof st));
    const char *nm[6] = {"start", "bits->lds", "walsh1", "x lw_fold", "walsh2", "rowinfo out"};
    for (int i = 1; i < 6; ++i) printf("  %-12s %6.2f us\n", nm[i], (st[i] - st[0]) * 0.01);
    return 0;
}
