// Host-overhead probe (development tool): rs_encode_device / rs_decode_device
// called from a C++ loop, to compare with the Python bench's per-step time.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/rs_mi355x.h"

int main(int argc, char **argv) {
    const uint64_t N = argc > 1 ? atoll(argv[1]) : 1024, M = argc > 2 ? atoll(argv[2]) : 1024,
                   S = argc > 3 ? atoll(argv[3]) : 1024;
    const int iters = 2000;
    rs_context *ctx = nullptr;
    if (rs_context_create(0, &ctx) != RS_OK) return 1;
    void *orig, *rec, *out;
    hipMalloc(&orig, N * S);
    hipMalloc(&rec, M * S);
    hipMalloc(&out, N * S);
    hipMemset(orig, 0x5a, N * S);
    rs_error err;
    for (int i = 0; i < 20; ++i) rs_encode_device(ctx, RS_RATE_DEFAULT, N, M, S, orig, rec, nullptr, &err);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto t0 = std::chrono::steady_clock::now();
    hipEventRecord(a, nullptr);
    for (int i = 0; i < iters; ++i) rs_encode_device(ctx, RS_RATE_DEFAULT, N, M, S, orig, rec, nullptr, &err);
    hipEventRecord(b, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    printf("encode %llu:%llu x %llu: %.2f us/encode (GPU), host enqueue %.2f us/encode, %.1f GiB/s\n",
           (unsigned long long)N, (unsigned long long)M, (unsigned long long)S, ms * 1000 / iters, host_us,
           double((N + M) * S) / (ms * 1e-3 / iters) / (1ull << 30));
    std::vector<uint8_t> op(N, 1), rp(M, 1);
    for (uint64_t i = 0; i < N && i < M; ++i) op[i] = 0;  // 100% loss
    for (int i = 0; i < 20; ++i)
        rs_decode_device(ctx, RS_RATE_DEFAULT, N, M, S, orig, op.data(), rec, rp.data(), out, nullptr, &err);
    hipDeviceSynchronize();
    t0 = std::chrono::steady_clock::now();
    hipEventRecord(a, nullptr);
    for (int i = 0; i < iters / 4; ++i)
        rs_decode_device(ctx, RS_RATE_DEFAULT, N, M, S, orig, op.data(), rec, rp.data(), out, nullptr, &err);
    hipEventRecord(b, nullptr);
    t1 = std::chrono::steady_clock::now();
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("decode 100%%: %.2f us/decode (GPU), host enqueue %.2f us\n", ms * 4000 / iters,
           std::chrono::duration<double, std::micro>(t1 - t0).count() * 4 / iters);
    rs_context_destroy(ctx);
    return 0;
}
