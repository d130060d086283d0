// VALU issue-rate probe (development tool): cycles per wave-instruction of
// v_lshrrev_b64 vs v_lshrrev_b32 vs v_perm_b32 with one and four waves per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int OP>
__global__ void k_rate(uint64_t *out, int iters) {
    uint64_t a = threadIdx.x, b = a * 3, c = a * 5, d = a * 7;
    uint32_t e = threadIdx.x, f = e * 3, g = e * 5, h = e * 7;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (OP == 0) {
                asm volatile("v_lshrrev_b64 %0, 3, %0\n v_lshrrev_b64 %1, 3, %1\n v_lshrrev_b64 %2, 3, %2\n v_lshrrev_b64 %3, 3, %3"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
            } else if constexpr (OP == 1) {
                asm volatile("v_lshrrev_b32 %0, 3, %0\n v_lshrrev_b32 %1, 3, %1\n v_lshrrev_b32 %2, 3, %2\n v_lshrrev_b32 %3, 3, %3"
                             : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
            } else if constexpr (OP == 2) {
                asm volatile("v_perm_b32 %0, %1, %2, %3\n v_perm_b32 %1, %2, %3, %0\n v_perm_b32 %2, %3, %0, %1\n v_perm_b32 %3, %0, %1, %2"
                             : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
            } else if constexpr (OP == 3) {
                asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96\n v_bitop3_b32 %1, %2, %3, %0 bitop3:0x96\n v_bitop3_b32 %2, %3, %0, %1 bitop3:0x96\n v_bitop3_b32 %3, %0, %1, %2 bitop3:0x96"
                             : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
            } else {  // a v_perm / v_bitop3 / v_and mix, as in a butterfly
                asm volatile("v_perm_b32 %0, %1, %2, %3\n v_bitop3_b32 %1, %2, %3, %0 bitop3:0x96\n v_and_b32 %2, %3, %0\n v_perm_b32 %3, %0, %1, %2"
                             : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (a + b + c + d + e + f + g + h == 12345) out[1000] = 1;
}

int main() {
    uint64_t *d;
    (void)hipMalloc(&d, 8 * 2048);
    const int iters = 1000;
    const char *names[5] = {"v_lshrrev_b64", "v_lshrrev_b32", "v_perm_b32", "v_bitop3_b32", "perm/bitop3/and"};
    for (int waves : {1, 4, 8, 16}) {
        for (int op = 0; op < 5; ++op) {
            auto launch = [&] {
                if (op == 0) k_rate<0><<<1, 64 * waves>>>(d, iters);
                else if (op == 1) k_rate<1><<<1, 64 * waves>>>(d, iters);
                else if (op == 2) k_rate<2><<<1, 64 * waves>>>(d, iters);
                else if (op == 3) k_rate<3><<<1, 64 * waves>>>(d, iters);
                else k_rate<4><<<1, 64 * waves>>>(d, iters);
            };
            launch();
            (void)hipDeviceSynchronize();
            launch();
            uint64_t cyc;
            (void)hipMemcpy(&cyc, d, 8, hipMemcpyDeviceToHost);
            // s_memtime counts at the shader clock; per wave-instruction on its SIMD
            const double per = double(cyc) / (iters * 32.0) / ((waves + 3) / 4);
            printf("%-14s waves/CU %2d: %.2f clk per wave-instruction per SIMD\n", names[op], waves, per);
        }
    }
    return 0;
}
