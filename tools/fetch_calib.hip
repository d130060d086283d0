// FETCH_SIZE calibration (development tool, MI355X_MICROARCH.md "HBM": access
// widths other than 16 B/lane streaming reads are uncalibrated).  Two kernels
// read a 512 MiB buffer (beyond the 256 MiB Infinity Cache) exactly once:
//   k_stream: 16 B per lane, fully coalesced (the guide's calibrated case)
//   k_packs : the column kernel's row access -- lanes 2k / 2k+1 read the low /
//             high 4-byte word of one 8-byte pack of a 64-byte block; the 8
//             workgroups that share a block run on one XCD (b % 8 mapping)
// Run: rocprofv3 --pmc FETCH_SIZE -- tools/_build/fetch_calib ; compare the
// per-dispatch FETCH_SIZE (KiB) with the 512 MiB read.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = size_t(512) << 20;

__global__ void k_stream(const uint4 *__restrict__ p, size_t n, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// rows of 1 KiB (16 blocks = 128 packs); a workgroup (512 threads, 2 rows per
// lane pair like the column kernel at n = 1024) reads one pack of 1024 rows.
__global__ void __launch_bounds__(512) k_packs(const uint8_t *__restrict__ p, uint32_t groups, uint32_t *out) {
    const uint32_t b = blockIdx.x;
    const uint32_t per_xcd = gridDim.x / 8;
    const uint32_t w = (b & 7u) * per_xcd + (b >> 3);  // XCD-aware, as k_mono
    const uint32_t group = w / 128, pk = w % 128;       // 1024 rows x 1 KiB per group
    if (group >= groups) return;
    const uint8_t *base = p + size_t(group) * (1024u * 1024u) + (pk >> 3) * 64u + (pk & 7u) * 4u;
    const uint32_t lane = threadIdx.x & 63u, half = (lane & 1u) * 32u;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t row = (threadIdx.x >> 1) + 256u * j;
        acc ^= *reinterpret_cast<const uint32_t *>(base + size_t(row) * 1024u + half);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kBytes);
    (void)hipDeviceSynchronize();
    k_stream<<<4096, 256>>>(reinterpret_cast<const uint4 *>(buf), kBytes / 16, out);
    const uint32_t groups = uint32_t(kBytes >> 20);
    k_packs<<<groups * 128, 512>>>(buf, groups, out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("fetch_calib: each kernel read %zu bytes once\n", kBytes);
    return 0;
}
