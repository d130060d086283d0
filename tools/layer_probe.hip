// Butterfly-layer latency probe (development tool): ns per layer of the column
// kernels' layer bodies, one workgroup per CU (256), NL dependent layers per lane:
//   V0  k_mono form: 2 rows per lane, gf_muladd2 (rs_gf.hpp) with a 16-word table read
//       from LDS (4 x ds_read_b128, 2 layers ahead), then the 2x2 register/lane
//       transpose on the next lane bit (rs_mono.hip xpose)
//   V1  k_lane form (rs_lane.hip): 1 row per lane, half products, 2 exchanges,
//       8 table words from LDS (2 x ds_read_b128)
//   V2 / V3  V0 / V1 with the tables in registers (no LDS reads)
//   V4  V0 without the transposes (register-bit layers only)
//   V5  V1 with lane bits 0, 1, 3 only (DPP; no permlane, no two-move bit 2)
// Usage: tools/_probe/layer_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../reed-solomon-simd_amd/csrc/rs_gf.hpp"

using namespace rs;

template <int J>
__device__ __forceinline__ void xp(uint32_t &a, uint32_t &b, uint32_t lane) {
    if constexpr (J == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    } else if constexpr (J == 5) {
        const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    } else {
        const bool up = (lane >> J) & 1u;
        const uint32_t recv = xor_lane<J>(up ? a : b);
        if (up) a = recv;
        else b = recv;
    }
}
__device__ __forceinline__ uint32_t half2(uint32_t x, uint32_t sh, const uint32_t (&t)[8]) {
    const uint32_t xr = __builtin_amdgcn_alignbit(x, x, 16);
    const uint64_t xx = (uint64_t(xr) << 32) | x;
    const uint64_t s0 = xx >> sh, s2 = xx >> (sh + 2u);
    constexpr uint32_t M = 0x03030303u, C = 0x04040000u;
    auto sel = [](uint32_t v) { return __builtin_amdgcn_bitop3_b32(v, M, C, 0xEA); };
    return xor3(__builtin_amdgcn_perm(t[1], t[0], sel(uint32_t(s0))), __builtin_amdgcn_perm(t[3], t[2], sel(uint32_t(s0 >> 32))),
                __builtin_amdgcn_perm(t[5], t[4], sel(uint32_t(s2)))) ^
           __builtin_amdgcn_perm(t[7], t[6], sel(uint32_t(s2 >> 32)));
}
template <int J>
__device__ __forceinline__ uint32_t partner(uint32_t v, uint32_t rm) {
    if constexpr (J == 4 || J == 5) {
        const auto r = J == 4 ? __builtin_amdgcn_permlane16_swap(v, v, false, false)
                              : __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (r[0] & rm) | (r[1] & ~rm);
    } else {
        return xor_lane<J>(v);
    }
}

constexpr int NL = 240;  // layers per lane (multiple of 6 and of the unroll)

template <int V, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) k_layers(uint32_t *out, const uint32_t *tabs) {
    __shared__ uint4 lds[1024];  // 256 tables of 64 B
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = reinterpret_cast<const uint4 *>(tabs)[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t a = threadIdx.x * 0x9E3779B9u, b = a ^ 0x5bd1e995u;
    uint32_t rm[6], sh[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        rm[j] = 0u - ((lane >> j) & 1u);
        sh[j] = ((lane >> j) & 1u) << 2;
    }
    uint32_t treg[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) treg[q] = tabs[q * 7 + (threadIdx.x & 15)];
    constexpr bool LDS = V == 0 || V == 1 || V == 4 || V == 5;
    constexpr bool HALF = V == 1 || V == 3 || V == 5;
    constexpr int NW = HALF ? 8 : 16;
    uint32_t tb[2][16];
    auto request = [&](int k) {
        const uint32_t slot = ((k * 37u) + (lane >> 1)) & 255u;
        const uint4 *p = lds + slot * 4u + (HALF ? (lane & 1u) * 2u : 0u);
#pragma unroll
        for (int q = 0; q < NW / 4; ++q) {
            const uint4 x = p[q];
            tb[k & 1][4 * q] = x.x, tb[k & 1][4 * q + 1] = x.y, tb[k & 1][4 * q + 2] = x.z, tb[k & 1][4 * q + 3] = x.w;
        }
    };
    if constexpr (LDS) {
        request(0);
        request(1);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NL; it += 6) {
        static_for<0, 6>([&](auto jc) {
            constexpr int J0 = decltype(jc)::value;
            constexpr int J = V == 5 ? (J0 % 3 == 2 ? 3 : J0 % 3) : J0;
            const int k = it + J0;
            uint32_t t[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = LDS ? tb[k & 1][q % NW] : treg[q] ^ uint32_t(k);
            if constexpr (!HALF) {
                ifft_bfly2(a, b, t);
                if constexpr (V != 4) xp<J>(a, b, lane);
            } else {
                const uint32_t p = partner<J>(a, rm[J]);
                const uint32_t bn = a ^ p;
                uint32_t t8[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) t8[q] = t[q];
                const uint32_t h = half2(bn, sh[J], t8);
                const uint32_t full = h ^ partner<J>(h, rm[J]);
                a = (bn & rm[J]) | ((a ^ full) & ~rm[J]);
            }
            if constexpr (LDS) request(k + 2);
        });
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63u) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = uint32_t(t1 - t0);
    if (a + b == 0x12345678u) out[100000] = a;
}

template <int V, int WAVES>
void run(const char *name, uint32_t *d_out, const uint32_t *d_tabs) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k_layers<V, WAVES><<<256, 64 * WAVES>>>(d_out, d_tabs);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) k_layers<V, WAVES><<<256, 64 * WAVES>>>(d_out, d_tabs);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint32_t cyc[16];
    (void)hipMemcpy(cyc, d_out, 64, hipMemcpyDeviceToHost);
    printf("%-34s waves/WG %2d: %6.1f ns per layer (events), %6.1f memtime clk per layer (wave 0)\n", name, WAVES,
           ms * 1e6 / reps / NL, double(cyc[0]) / NL);
}

int main() {
    uint32_t *d_out, *d_tabs;
    (void)hipMalloc(&d_out, 4 * 200000);
    (void)hipMalloc(&d_tabs, 16384);
    uint32_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = uint32_t(i) * 2654435761u;
    (void)hipMemcpy(d_tabs, h, 16384, hipMemcpyHostToDevice);
    run<0, 8>("V0 mono form (LDS, transposes)", d_out, d_tabs);
    run<0, 16>("V0 mono form (LDS, transposes)", d_out, d_tabs);
    run<1, 8>("V1 lane form (LDS)", d_out, d_tabs);
    run<1, 16>("V1 lane form (LDS)", d_out, d_tabs);
    run<2, 8>("V2 mono form, register tables", d_out, d_tabs);
    run<2, 16>("V2 mono form, register tables", d_out, d_tabs);
    run<3, 8>("V3 lane form, register tables", d_out, d_tabs);
    run<3, 16>("V3 lane form, register tables", d_out, d_tabs);
    run<4, 8>("V4 mono form, no transposes", d_out, d_tabs);
    run<4, 16>("V4 mono form, no transposes", d_out, d_tabs);
    run<5, 8>("V5 lane form, DPP bits only", d_out, d_tabs);
    run<5, 16>("V5 lane form, DPP bits only", d_out, d_tabs);
    run<0, 4>("V0 mono form (LDS, transposes)", d_out, d_tabs);
    run<1, 4>("V1 lane form (LDS)", d_out, d_tabs);
    run<2, 4>("V2 mono form, register tables", d_out, d_tabs);
    run<0, 1>("V0 mono form (LDS, transposes)", d_out, d_tabs);
    run<2, 1>("V2 mono form, register tables", d_out, d_tabs);
    run<4, 1>("V4 mono form, no transposes", d_out, d_tabs);
    return 0;
}
