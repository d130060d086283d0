// VALU issue rate per instruction kind (development tool): every lane of
// 256 workgroups x W waves runs 8 independent chains of one instruction kind
// (inline asm, 8 x 16 instructions per loop trip), so the time measures issue
// throughput, not latency.  Prints clocks (at 2.4 GHz) per wave64 instruction
// per SIMD for each kind and wave count.  Which instructions of the GF multiply
// mix (rs_gf.hpp gf_muladd2 / gf_muladd4) are the costly ones?
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/_probe/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../reed-solomon-simd_amd/csrc/rs_gf.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

#define R8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
#define REP16(x) x x x x x x x x x x x x x x x x

// one kind: OP(i) is the asm text of chain i's instruction; a..h are the 8 chain registers
#define KIND(name, body)                                                                   \
    __global__ void __launch_bounds__(1024) name(uint32_t *out, int iters, uint32_t s) { \
        uint32_t a = threadIdx.x ^ s, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 9u, f = a * 11u, g = a * 13u, \
                 h = a * 15u;                                                              \
        const uint32_t k1 = s | 0x03030303u, k2 = s ^ 0x04040000u;                          \
        for (int it = 0; it < iters; ++it) {                                               \
            body                                                                           \
        }                                                                                  \
        if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 0x12345678u) out[threadIdx.x] = a;           \
    }

#define OP3(ins, r) asm volatile(ins " %0, %0, %1, %2" : "+v"(r) : "v"(k1), "v"(k2));
#define OP2(ins, r) asm volatile(ins " %0, %0, %1" : "+v"(r) : "v"(k1));
#define BODY3(ins) REP16(OP3(ins, a) OP3(ins, b) OP3(ins, c) OP3(ins, d) OP3(ins, e) OP3(ins, f) OP3(ins, g) OP3(ins, h))
#define BODY2(ins) REP16(OP2(ins, a) OP2(ins, b) OP2(ins, c) OP2(ins, d) OP2(ins, e) OP2(ins, f) OP2(ins, g) OP2(ins, h))

KIND(k_perm, BODY3("v_perm_b32"))
KIND(k_xor2, BODY2("v_xor_b32"))
KIND(k_and2, BODY2("v_and_b32"))
KIND(k_andor, BODY3("v_and_or_b32"))
KIND(k_alignbit, BODY3("v_alignbit_b32"))
KIND(k_bfe, BODY3("v_bfe_u32"))
KIND(k_lshlor, BODY3("v_lshl_or_b32"))
#define OPB(r)                                          \
    r = __builtin_amdgcn_bitop3_b32(r, k1, k2, 0xEA); \
    asm volatile("" : "+v"(r));
KIND(k_bitop3, REP16(OPB(a) OPB(b) OPB(c) OPB(d) OPB(e) OPB(f) OPB(g) OPB(h)))
// 64-bit shift: 4 chains of register pairs
#define OPS64(r)                                                                   \
    {                                                                              \
        uint64_t t = (uint64_t(r) << 32) | k1;                                     \
        asm volatile("v_lshrrev_b64 %0, 2, %0" : "+v"(t));                         \
        r = uint32_t(t) ^ uint32_t(t >> 32);                                       \
    }
#define OPL64(r) asm volatile("v_lshrrev_b64 %0, 2, %0" : "+v"(r));
__global__ void __launch_bounds__(1024) k_lshr64(uint32_t *out, int iters, uint32_t s) {
    uint64_t a = threadIdx.x ^ s, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 9u, f = a * 11u, g = a * 13u,
             h = a * 15u;
    for (int it = 0; it < iters; ++it) {
        REP16(OPL64(a) OPL64(b) OPL64(c) OPL64(d) OPL64(e) OPL64(f) OPL64(g) OPL64(h))
    }
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 0x12345678u) out[threadIdx.x] = uint32_t(a);
}
// DPP move (row_shl:1) and a permlane32 swap
#define OPD(r) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r));
KIND(k_dpp, REP16(OPD(a) OPD(b) OPD(c) OPD(d) OPD(e) OPD(f) OPD(g) OPD(h)))
#define OPXD(r) asm volatile("v_xor_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k1));
KIND(k_xordpp, REP16(OPXD(a) OPXD(b) OPXD(c) OPXD(d) OPXD(e) OPXD(f) OPXD(g) OPXD(h)))
#define OPPL(r, q) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(r), "+v"(q));
KIND(k_pl32, REP16(OPPL(a, b) OPPL(c, d) OPPL(e, f) OPPL(g, h) OPPL(a, b) OPPL(c, d) OPPL(e, f) OPPL(g, h)))

// The multiply mixes themselves: 8 independent gf_muladd2 chains (24 VALU each),
// 4 independent gf_muladd4 chains (26 VALU each); tables in registers
__global__ void __launch_bounds__(1024) k_mul2(uint32_t *out, int iters, uint32_t s) {
    uint32_t t[16], x[8];
    for (int i = 0; i < 16; ++i) t[i] = (threadIdx.x + i) * 0x01010101u ^ s;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * (i + 3);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t acc = x[(i + 1) & 7];
                rs::gf_muladd2(acc, x[i], t);
                x[i] = acc;
                asm volatile("" : "+v"(x[i]));
            }
    }
    uint32_t z = 0;
    for (int i = 0; i < 8; ++i) z ^= x[i];
    if (z == 0x12345678u) out[threadIdx.x] = z;
}
__global__ void __launch_bounds__(1024) k_mul4(uint32_t *out, int iters, uint32_t s) {
    uint32_t t[20], xl[4], xh[4];
    for (int i = 0; i < 20; ++i) t[i] = (threadIdx.x + i) * 0x01010101u ^ s;
    for (int i = 0; i < 4; ++i) xl[i] = threadIdx.x * (i + 3), xh[i] = threadIdx.x * (i + 7);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t al = xl[(i + 1) & 3], ah = xh[(i + 1) & 3];
                rs::gf_muladd4(al, ah, xl[i], xh[i], t);
                xl[i] = al, xh[i] = ah;
                asm volatile("" : "+v"(xl[i]), "+v"(xh[i]));
            }
    }
    uint32_t z = 0;
    for (int i = 0; i < 4; ++i) z ^= xl[i] ^ xh[i];
    if (z == 0x12345678u) out[threadIdx.x] = z;
}

typedef void (*Kern)(uint32_t *, int, uint32_t);

int main() {
    uint32_t *out;
    CK(hipMalloc(&out, 4096));
    struct {
        const char *name;
        Kern k;
    } kinds[] = {{"v_perm_b32", k_perm},       {"v_xor_b32", k_xor2},         {"v_and_b32", k_and2},
                 {"v_and_or_b32", k_andor},     {"v_alignbit_b32", k_alignbit},
                 {"v_bfe_u32", k_bfe},         {"v_lshl_or_b32", k_lshlor},   {"v_bitop3_b32", k_bitop3},
                 {"v_lshrrev_b64", k_lshr64},  {"v_mov_b32_dpp", k_dpp},      {"v_xor_b32_dpp", k_xordpp},
                 {"v_permlane32_swap", k_pl32}, {"gf_muladd2 (/24)", k_mul2}, {"gf_muladd4 (/26)", k_mul4}};
    const int iters = 2000;
    // instructions per loop trip (per lane): 128; the multiply mixes 16 x 24 = 384, 16 x 26 = 416
    auto per_trip_of = [](Kern k) { return k == k_mul2 ? 384 : k == k_mul4 ? 416 : 128; };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &kd : kinds) {
        printf("%-18s", kd.name);
        for (int waves : {1, 2, 4, 8}) {  // waves per SIMD: 256 workgroups (one per CU) x 4 * waves
            const int threads = 64 * 4 * waves;
            kd.k<<<256, threads>>>(out, 10, 1);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            kd.k<<<256, threads>>>(out, iters, 1);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            // wave-instructions per SIMD: waves * iters * per_trip
            const double clocks = ms * 1e-3 * 2.4e9 / (double(waves) * iters * per_trip_of(kd.k));
            printf("  %d w/SIMD %5.2f clk", waves, clocks);
        }
        printf("\n");
    }
    return 0;
}
