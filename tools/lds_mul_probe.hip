// Price of an LDS-table GF(2^16) multiply against the v_perm_b32 multiply
// (development tool; VERDICT r05 item 5, north_star's "LDS-staged log/exp tables").
//
// Every lane of 256 workgroups (one per CU) x W waves per SIMD keeps 4 independent
// 4-element packs and runs, per loop trip, NT = 8 wave-uniform multipliers over all
// 4 packs (acc ^= x * m, the butterfly's multiply-add), so the time measures
// throughput.  Forms (all multiply by the same 8 constants, so their results must be
// bit-identical, and the probe checks that):
//   0 perm/lds   rs_gf.hpp gf_muladd4 (26 VALU per 4 elements), its 20-word table read
//                from LDS per multiplier (5 ds_read_b128, one address per wave: a
//                broadcast) -- what the pass kernels do
//   1 perm/regs  gf_muladd4, one table held in registers (the pure VALU bound; one
//                multiplier, so not compared)
//   2 byte/lds   x * m = TL[lo] ^ TH[hi]: two 256-entry tables per multiplier in LDS
//                (entry = product low byte | high byte << 16), 2 ds_read_b32 per
//                element at data-dependent addresses
//   3 nib/lds    four 16-entry nibble tables (the reference's Mul16, tables.rs:235-251,
//                engine_nosimd.rs:59-111), each replicated 4x across the banks so the
//                16 lanes of a quarter-wave hit one replica: a bank holds one entry of
//                one replica, lanes sharing a bank read the same word (broadcast, no
//                conflict); 4 ds_read_b32 per element
//   4 mixed      the low input bytes through v_perm (fields of the low plane, both
//                output planes), the high input bytes through the LDS byte table TH
// Output: clocks (2.4 GHz) per element per CU and elements per clock per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lds_mul_probe.hip
//          reed-solomon-simd_amd/csrc/gf_tables.cpp -o tools/_build/lds_mul_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../reed-solomon-simd_amd/csrc/gf_tables.hpp"
#include "../reed-solomon-simd_amd/csrc/rs_gf.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr int NT = 8;          // multipliers per loop trip (wave-uniform)
constexpr int PW = 20;         // perm table words
constexpr int BW = 512;        // byte tables: TL[256], TH[256]
constexpr int NW = 4 * 4 * 16; // nibble tables: 4 fields x 4 replicas x 16 entries

using rs::xor3;

__device__ __forceinline__ void mul_byte(uint32_t &al, uint32_t &ah, uint32_t xl, uint32_t xh, const uint32_t *T) {
    uint32_t p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = T[(xl >> (8 * j)) & 255u] ^ T[256 + ((xh >> (8 * j)) & 255u)];
    const uint32_t w01 = p[0] | (p[1] << 8), w23 = p[2] | (p[3] << 8);  // [lo0 lo1 hi0 hi1], [lo2 lo3 hi2 hi3]
    al ^= __builtin_amdgcn_perm(w23, w01, 0x05040100u);
    ah ^= __builtin_amdgcn_perm(w23, w01, 0x07060302u);
}

__device__ __forceinline__ void mul_nib(uint32_t &al, uint32_t &ah, uint32_t xl, uint32_t xh, const uint32_t *T,
                                        uint32_t rep) {
    uint32_t p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t lo = (xl >> (8 * j)) & 255u, hi = (xh >> (8 * j)) & 255u;
        p[j] = xor3(T[(0 * 4 + rep) * 16 + (lo & 15u)], T[(1 * 4 + rep) * 16 + (lo >> 4)],
                    T[(2 * 4 + rep) * 16 + (hi & 15u)]) ^
               T[(3 * 4 + rep) * 16 + (hi >> 4)];
    }
    const uint32_t w01 = p[0] | (p[1] << 8), w23 = p[2] | (p[3] << 8);
    al ^= __builtin_amdgcn_perm(w23, w01, 0x05040100u);
    ah ^= __builtin_amdgcn_perm(w23, w01, 0x07060302u);
}

__device__ __forceinline__ void mul_mixed(uint32_t &al, uint32_t &ah, uint32_t xl, uint32_t xh, const uint32_t *t,
                                          const uint32_t *TH) {
    // low input bytes: gf_muladd4's low-plane fields (tables words 0-4 low out, 5-9 high out)
    const uint32_t l0 = xl & 0x07070707u, l1 = (xl >> 3) & 0x07070707u, l2 = (xl >> 6) & 0x03030303u;
    const uint32_t la = xor3(__builtin_amdgcn_perm(t[1], t[0], l0), __builtin_amdgcn_perm(t[3], t[2], l1),
                             __builtin_amdgcn_perm(t[4], t[4], l2));
    const uint32_t ha = xor3(__builtin_amdgcn_perm(t[6], t[5], l0), __builtin_amdgcn_perm(t[8], t[7], l1),
                             __builtin_amdgcn_perm(t[9], t[9], l2));
    // high input bytes: the byte table
    uint32_t p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = TH[(xh >> (8 * j)) & 255u];
    const uint32_t w01 = p[0] | (p[1] << 8), w23 = p[2] | (p[3] << 8);
    al = xor3(al, la, __builtin_amdgcn_perm(w23, w01, 0x05040100u));
    ah = xor3(ah, ha, __builtin_amdgcn_perm(w23, w01, 0x07060302u));
}

template <int KIND>
__global__ void __launch_bounds__(1024) k_probe(const uint32_t *gperm, const uint32_t *gbyte, const uint32_t *gnib,
                                                uint32_t *out, int iters) {
    __shared__ uint32_t sperm[NT * PW];
    __shared__ uint32_t sbyte[NT * BW];
    __shared__ uint32_t snib[NT * NW];
    for (uint32_t i = threadIdx.x; i < NT * PW; i += blockDim.x) sperm[i] = gperm[i];
    for (uint32_t i = threadIdx.x; i < NT * BW; i += blockDim.x) sbyte[i] = gbyte[i];
    for (uint32_t i = threadIdx.x; i < NT * NW; i += blockDim.x) snib[i] = gnib[i];
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t xl[4], xh[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t h = gid * 0x9E3779B1u + uint32_t(i) * 0x85EBCA77u;
        h ^= h >> 15;
        h *= 0x2C1B3C6Du;
        xl[i] = h;
        h ^= h >> 13;
        h *= 0x297A2D39u;
        xh[i] = h ^ (h >> 16);
    }
    const uint32_t rep = (threadIdx.x >> 4) & 3u;
    uint32_t treg[PW];
    if constexpr (KIND == 1)
#pragma unroll
        for (int q = 0; q < PW; ++q) treg[q] = sperm[q];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < NT; ++m) {
            // every trip re-reads the tables (no form may hoist its table reads out of
            // the loop), at compile-time LDS offsets (the byte tables' addresses are
            // then one v_lshlrev_b32_sdwa per lookup)
            asm volatile("" ::: "memory");
            uint32_t t[PW];
            if constexpr (KIND == 0 || KIND == 4) {
#pragma unroll
                for (int q = 0; q < PW / 4; ++q) {
                    const uint4 v = reinterpret_cast<const uint4 *>(sperm + m * PW)[q];
                    t[4 * q] = v.x, t[4 * q + 1] = v.y, t[4 * q + 2] = v.z, t[4 * q + 3] = v.w;
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t al = xl[(i + 1) & 3], ah = xh[(i + 1) & 3];
                if constexpr (KIND == 0) rs::gf_muladd4(al, ah, xl[i], xh[i], t);
                else if constexpr (KIND == 1) rs::gf_muladd4(al, ah, xl[i], xh[i], treg);
                else if constexpr (KIND == 2) mul_byte(al, ah, xl[i], xh[i], sbyte + m * BW);
                else if constexpr (KIND == 3) mul_nib(al, ah, xl[i], xh[i], snib + m * NW, rep);
                else mul_mixed(al, ah, xl[i], xh[i], t, sbyte + m * BW + 256);
                xl[i] = al, xh[i] = ah;
            }
        }
    }
    uint32_t zl = 0, zh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) zl ^= xl[i] * (2u * i + 1u), zh ^= xh[i] * (2u * i + 3u);
    out[2 * gid] = zl;
    out[2 * gid + 1] = zh;
}

typedef void (*Kern)(const uint32_t *, const uint32_t *, const uint32_t *, uint32_t *, int);

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const rs::GfTables &T = rs::tables();
    // 8 multipliers: log_m spread over the field (none is 65535: every one multiplies)
    const uint16_t logs[NT] = {1, 777, 4242, 12345, 23456, 34567, 45678, 65000};
    std::vector<uint32_t> perm(NT * PW), byte(NT * BW), nib(NT * NW);
    for (int m = 0; m < NT; ++m) {
        std::memcpy(&perm[m * PW], &T.perm_by_log[size_t(logs[m]) * rs::kPermWords], PW * 4);
        for (uint32_t b = 0; b < 256; ++b) {
            const uint16_t pl = T.mul(uint16_t(b), logs[m]), ph = T.mul(uint16_t(b << 8), logs[m]);
            byte[m * BW + b] = (pl & 0xFFu) | (uint32_t(pl >> 8) << 16);
            byte[m * BW + 256 + b] = (ph & 0xFFu) | (uint32_t(ph >> 8) << 16);
        }
        for (int f = 0; f < 4; ++f)
            for (int r = 0; r < 4; ++r)
                for (uint32_t v = 0; v < 16; ++v) {
                    const uint16_t p = T.mul(uint16_t(v << (4 * f)), logs[m]);
                    nib[m * NW + (f * 4 + r) * 16 + v] = (p & 0xFFu) | (uint32_t(p >> 8) << 16);
                }
    }
    uint32_t *d_perm, *d_byte, *d_nib, *d_out;
    CK(hipMalloc(&d_perm, perm.size() * 4));
    CK(hipMalloc(&d_byte, byte.size() * 4));
    CK(hipMalloc(&d_nib, nib.size() * 4));
    const size_t max_threads = 256 * 1024;
    CK(hipMalloc(&d_out, max_threads * 8));
    CK(hipMemcpy(d_perm, perm.data(), perm.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_byte, byte.data(), byte.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_nib, nib.data(), nib.size() * 4, hipMemcpyHostToDevice));
    struct {
        const char *name;
        Kern k;
    } kinds[] = {{"0 perm/lds (gf_muladd4)", k_probe<0>}, {"1 perm/regs (1 table)", k_probe<1>},
                 {"2 byte/lds", k_probe<2>},              {"3 nib/lds x4 replicas", k_probe<3>},
                 {"4 mixed perm+byte/lds", k_probe<4>}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("# tools/lds_mul_probe.hip: 256 workgroups x 4W waves, %d trips x %d multipliers x 4 packs x 4 elements "
           "per lane; clk = 2.4 GHz clocks per element per CU (lower is better)\n", iters, NT);
    int bad = 0;
    for (int waves : {1, 2, 4}) {
        const int threads = 256 * waves;
        std::vector<uint32_t> ref;
        for (auto &kd : kinds) {
            kd.k<<<256, threads>>>(d_perm, d_byte, d_nib, d_out, 2);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            kd.k<<<256, threads>>>(d_perm, d_byte, d_nib, d_out, iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<uint32_t> got(size_t(256) * threads * 2);
            CK(hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost));
            const char *check = "";
            if (kd.k != kinds[1].k) {
                if (ref.empty()) ref = got;
                else if (got != ref) check = "  MISMATCH", ++bad;
                else check = "  (= form 0)";
            }
            const double elems_per_cu = double(threads) * iters * NT * 16;
            const double clk = ms * 1e-3 * 2.4e9 / elems_per_cu;
            printf("%d w/SIMD  %-26s %8.3f ms  %6.3f clk/elem/CU  %6.2f elem/clk/CU%s\n", waves, kd.name, ms, clk,
                   1.0 / clk, check);
        }
    }
    return bad ? 1 : 0;
}
