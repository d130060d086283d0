// Lane column kernel ("k_lane") of the MI355X Reed-Solomon engine: the
// single-chunk encode of 2^L rows, 8 <= L <= 10, with ONE row per lane.
//
// Like k_mono (rs_mono.hip), one workgroup owns every row of one 2-element
// pack (elements 2p, 2p + 1 of every shard: one word [lo0 lo1 hi0 hi1] per row,
// reference block layout src/algorithm.md:18-31), and runs the whole encode --
// IFFT (src/engine/engine_naive.rs:75-105) then FFT (:43-73), HighRate
// (src/rate/rate_high.rs:44-87) or LowRate (src/rate/rate_low.rs:44-87), one
// chunk -- with no cross-workgroup hand-off.  k_mono holds 2 rows per lane: a
// 2^10-row column is 512 threads, 2 waves per SIMD, and a wave issues one VALU
// instruction per ~5.8 clocks at best (tools/valu_probe.hip), so
// the 20 layers ran at ~2 waves' issue rate.  Here a column is 2^L threads
// (4 waves per SIMD at L = 10) and the two lanes of a butterfly split its
// multiply: each computes the partial product of two of the four 2-bit fields
// of gf_muladd2 (rs_gf.hpp) from half of the 16-word table, and one DPP /
// permlane exchange completes it.  Per layer a lane issues ~22 VALU against
// ~30 + transposes for a 2-row lane, and reads 32 bytes of table from LDS.
//
// Placements (row index bits): A = lane bits 0..5, wave bits 6..L-1 (a wave
// holds 64 consecutive rows); B = lane bits L-6..L-1, wave bits 0..L-7.
//   IFFT layers 0..5 in A (wave-private tables), one LDS remap,
//   IFFT layers 6..L-1 and FFT layers L-1..L-6 in B (tables shared by the waves),
//   one LDS remap, FFT layers L-7..0 in A (wave-private tables).
// Every table of the launch is staged in LDS at the start, built from its 8-word
// basis (rs_codec.cpp basis_images, rs_gf.hpp basis2_expand): 16-byte pieces,
// piece-major per region (position piece * 68 + slot: the two lanes of a
// butterfly read pieces {0, 1} and {2, 3} of one table, 68 = 4 mod 16 spreads
// them over the banks).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>

#include "rs_device.hpp"
#include "rs_gf.hpp"

namespace rs {
namespace {

#ifdef RS_LANE_STAMPS  // tools/lane_probe.hip: per-workgroup timestamps of wave 0 and the last wave
__device__ uint64_t g_lane_stamps[4096][2][12];
#define RS_LSTAMP(i)                                                                                        \
    do {                                                                                                    \
        asm volatile("" ::: "memory");                                                                      \
        if ((threadIdx.x & 63u) == 0 && (threadIdx.x == 0 || threadIdx.x == blockDim.x - 64) && blockIdx.x < 4096) \
            g_lane_stamps[blockIdx.x][threadIdx.x ? 1 : 0][i] = __builtin_amdgcn_s_memrealtime();           \
    } while (0)
#else
#define RS_LSTAMP(i)
#endif

template <int L>
struct LaneGeo {
    static_assert(L >= 8 && L <= 10, "lane kernel: 2^8 .. 2^10 rows (one row per thread)");
    static constexpr int WB = L - 6;                        // wave bits
    static constexpr uint32_t n = 1u << L, W = 1u << WB;    // rows = threads, waves
    static constexpr uint32_t NT = 68;                      // slots per piece plane of a region (>= 63, = 4 mod 16)
    static constexpr uint32_t kRegion = 4 * NT * 16;        // bytes of a region (4 piece planes)
    static constexpr uint32_t kA1 = 63;                     // phase-A IFFT tables of a wave: layers 0..5
    static constexpr uint32_t kA3 = 64 - (64 >> WB);        // phase-A FFT tables of a wave: layers 0..WB-1
    static constexpr uint32_t kShI = (1u << WB) - 1;        // IFFT layers 6..L-1 (shared by the waves)
    static constexpr uint32_t kShF = (n >> WB) - 1;         // FFT layers WB..L-1 (= 63)
    // LDS (bytes): column plane | shared IFFT | shared FFT | W x phase-A IFFT | W x phase-A FFT
    static constexpr uint32_t kPlane = 4 * n;
    static constexpr uint32_t kShIBase = kPlane, kShFBase = kShIBase + kRegion;
    static constexpr uint32_t kA1Base = kShFBase + kRegion, kA3Base = kA1Base + W * kRegion;
    static constexpr uint32_t kBytes = kA3Base + W * kRegion;
    static_assert(kBytes <= 160 * 1024, "lane kernel: LDS per workgroup");
    static_assert(kShI <= NT && kShF <= NT, "shared regions");
};

// Row index bits -> LDS plane word, XOR-swizzled inside 32-word runs (both
// placements' accesses are conflict-free: see rs_mono.hip swz)
__device__ __forceinline__ uint32_t lswz(uint32_t r) { return r ^ ((r >> 5) & 31u); }

// Partial product of 2-element packs (gf_muladd2, rs_gf.hpp): sh = 0 forms the
// lookups of fields 0 and 1 (table words 0..7), sh = 4 those of fields 2 and 3
// (words 8..15); t = the lane's 8 words.  The XOR of the two partials is x * m.
__device__ __forceinline__ uint32_t gf_half2(uint32_t x, uint32_t sh, const uint32_t (&t)[8]) {
    const uint32_t xr = __builtin_amdgcn_alignbit(x, x, 16);
    const uint64_t xx = (uint64_t(xr) << 32) | x;
    const uint64_t s0 = xx >> sh, s2 = xx >> (sh + 2u);
    constexpr uint32_t M = 0x03030303u, C = 0x04040000u;
    auto sel = [](uint32_t v) { return __builtin_amdgcn_bitop3_b32(v, M, C, 0xEA); };
    const uint32_t a = __builtin_amdgcn_perm(t[1], t[0], sel(uint32_t(s0)));
    const uint32_t b = __builtin_amdgcn_perm(t[3], t[2], sel(uint32_t(s0 >> 32)));
    const uint32_t c = __builtin_amdgcn_perm(t[5], t[4], sel(uint32_t(s2)));
    const uint32_t d = __builtin_amdgcn_perm(t[7], t[6], sel(uint32_t(s2 >> 32)));
    return xor3(a, b, c) ^ d;
}

// The value of lane ^ 2^J (rm = the lane's role mask for bit J: all ones when
// the bit is set): DPP within rows of 16 lanes, v_permlane{16,32}_swap across them
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

// One butterfly layer on lane bit J (engine_naive.rs:64-68 / 96-100).  The
// lane with bit J clear holds a, its partner b; both form b' (IFFT) / b (FFT),
// each its half of the product, and exchange halves.  rm: all ones on the b lane.
template <int J, bool IFFT>
__device__ __forceinline__ void lane_layer(uint32_t &v, const uint32_t (&t)[8], uint32_t rm, uint32_t sh) {
    const uint32_t p = partner<J>(v, rm);
    if constexpr (IFFT) {  // b ^= a; a ^= b * m
        const uint32_t bn = v ^ p;
        const uint32_t h = gf_half2(bn, sh, t);
        const uint32_t full = h ^ partner<J>(h, rm);
        v = (bn & rm) | ((v ^ full) & ~rm);
    } else {  // a ^= b * m; b ^= a
        const uint32_t b = (v & rm) | (p & ~rm);
        const uint32_t h = gf_half2(b, sh, t);
        const uint32_t full = h ^ partner<J>(h, rm);
        v = xor3(v, full, p & rm);
    }
}

// The layer sequence: k-th layer of the kernel (0 .. 2L-1) -> row bit x, lane
// bit J, IFFT?, region (0 = phase-A IFFT, 1 = shared IFFT, 2 = shared FFT,
// 3 = phase-A FFT) and the layer's first slot in the region.
template <int L>
struct LaneSeq {
    static constexpr int WB = L - 6;
    static constexpr uint32_t n = 1u << L;
    static constexpr int bit(int k) { return k < L ? k : 2 * L - 1 - k; }
    static constexpr bool ifft(int k) { return k < L; }
    static constexpr int lane_bit(int k) { return (k < 6 || k >= 2 * L - WB) ? bit(k) : bit(k) - WB; }
    static constexpr int region(int k) { return k < 6 ? 0 : k < L ? 1 : k < 2 * L - WB ? 2 : 3; }
    static constexpr uint32_t slot0(int k) {
        const int x = bit(k);
        switch (region(k)) {
            case 0:
            case 3: return 64u - (64u >> x);
            case 1: return (n >> 6) - (n >> x);
            default: return (n >> WB) - (n >> x);
        }
    }
};

// 2x2 transpose of (word pair, lane bit 0): the even lane ends with (a, the odd
// lane's a), the odd lane with (the even lane's b, b) -- paired row I/O
__device__ __forceinline__ void pair_xpose(uint32_t &a, uint32_t &b, uint32_t lane) {
    const bool up = lane & 1u;
    const uint32_t recv = xor_lane<0>(up ? a : b);
    if (up) a = recv;
    else b = recv;
}

// Region slot t of a phase-A region (layers 0..5 / 0..WB-1) -> layer and group.
__device__ __forceinline__ uint32_t a_layer(uint32_t t) { return 6u - uint32_t(32 - __builtin_clz(63u - t)); }

template <int L, bool BATCH>
__global__ void __launch_bounds__(1 << L) k_lane(const MonoCore A) {
    using G = LaneGeo<L>;
    using Q = LaneSeq<L>;
    constexpr uint32_t n = G::n;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
    uint32_t *plane = reinterpret_cast<uint32_t *>(lds8);

    const uint32_t b = blockIdx.x;
    const uint32_t pk = (b & 7u) * A.packs_per_xcd + (b >> 3);  // XCD-aware, as k_mono
    if (pk >= A.packs) return;
    const uint8_t *src0 = A.src[0].base, *src1 = A.src[1].base;
    uint8_t *dst = const_cast<uint8_t *>(A.dst.base);
    if constexpr (BATCH) {
        src0 += uint64_t(blockIdx.y) * A.src_bstride[0];
        src1 += uint64_t(blockIdx.y) * A.src_bstride[1];
        dst += uint64_t(blockIdx.y) * A.dst_bstride;
    }
    const PackIO io = pack_io2(A.fmt, pk);
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t *img_i = A.img + uint64_t(A.ifft_img) * A.img_words;
    const uint32_t *img_f = A.img + uint64_t(A.fft_img) * A.img_words;
    RS_LSTAMP(0);

    // ---- row loads (placement A: row = tid), paired: lanes 2k, 2k+1 read the low and
    // the high half of one row in one instruction (one cache line per lane pair)
    const uint32_t off = io.lo + ((lane & 1u) ? io.hi_delta : 0u);
    const uint8_t *any_row = A.src[0].row_end > A.src[0].row_begin ? src0 : src1;
    uint32_t w[2], okm = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t r = (tid & ~1u) | uint32_t(j);
        const uint8_t *p = nullptr;
        if (r >= A.src[0].row_begin && r < A.src[0].row_end) p = src0 + uint64_t(r - A.src[0].row_begin) * A.src[0].stride;
        if (A.nsrc > 1 && r >= A.src[1].row_begin && r < A.src[1].row_end)
            p = src1 + uint64_t(r - A.src[1].row_begin) * A.src[1].stride;
        const uint8_t *a = (p ? p : any_row) + off;
        okm |= uint32_t(p != nullptr) << j;
        w[j] = io.bytes ? ld_half(a, io)
                        : *reinterpret_cast<const uint32_t *>(a - (reinterpret_cast<uintptr_t>(a) & 3u));
    }

    // ---- table staging loads: 16-byte pieces of the basis images (rs_codec.cpp
    // basis_images: 2 per table, slot-major), built into the table's 4 pieces while
    // written (basis2_expand; half the staging's L2 requests)
    // (RS_LANE_BASIS=0: the 16-word images, 4 pieces per table, copied as they are)
    constexpr uint32_t P = RS_LANE_BASIS ? 2 : 4;  // image pieces per table
    auto img_piece = [](const uint32_t *img, uint32_t slot, uint32_t piece) {
        return reinterpret_cast<const uint4 *>(img)[slot * P + piece];
    };
    // write image piece h of table slot s into the planes at `base` (basis piece h:
    // table pieces 2h, 2h + 1)
    auto put = [&](uint32_t base, uint32_t s, uint32_t h, const uint4 &v) {
        if constexpr (P == 2) {
            uint4 a, b;
            basis2_expand(v, a, b);
            *reinterpret_cast<uint4 *>(lds8 + base + ((2u * h) * G::NT + s) * 16u) = a;
            *reinterpret_cast<uint4 *>(lds8 + base + ((2u * h + 1u) * G::NT + s) * 16u) = b;
        } else {
            *reinterpret_cast<uint4 *>(lds8 + base + (h * G::NT + s) * 16u) = v;
        }
    };
    constexpr int K1 = (P * G::kA1 + 63) / 64, K3 = (P * G::kA3 + 63) / 64;
    constexpr uint32_t kShP = P * (G::kShI + G::kShF);
    constexpr int KS = (kShP + n - 1) / n;
    uint4 v1[K1], v3[K3], vs[KS];
    // phase-A regions: region slot t = layer x's first slot + g (g < 32 >> x) holds the
    // wave's group g of layer x: image slot n - (n >> x) + wave * (32 >> x) + g
#pragma unroll
    for (int k = 0; k < K1; ++k) {
        uint32_t q = lane + 64u * k;
        q = q < P * G::kA1 ? q : P * G::kA1 - 1;
        const uint32_t t = q / P, x = a_layer(t);
        v1[k] = img_piece(img_i, n - (n >> x) + wave * (32u >> x) + t - (64u - (64u >> x)), q % P);
    }
    // the shared and the phase-A FFT tables, also up front (requested during the
    // phase-A IFFT instead: 2^8 rows 4.35 -> 4.70 us, 2^9 5.50 -> 5.77 us, 2^10
    // unchanged; profiles/r05c/lane_probe.txt)
    {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            uint32_t q = tid + n * k;
            q = q < kShP ? q : kShP - 1;
            const uint32_t t = q / P;
            // shared IFFT: image slots n - n/64 .. (layers 6..L-1); shared FFT: n - n/2^WB ..
            vs[k] = t < G::kShI ? img_piece(img_i, n - (n >> 6) + t, q % P)
                                : img_piece(img_f, n - (n >> G::WB) + (t - G::kShI), q % P);
        }
#pragma unroll
        for (int k = 0; k < K3; ++k) {
            uint32_t q = lane + 64u * k;
            q = q < P * G::kA3 ? q : P * G::kA3 - 1;
            const uint32_t t = q / P, x = a_layer(t);
            v3[k] = img_piece(img_f, n - (n >> x) + wave * (32u >> x) + t - (64u - (64u >> x)), q % P);
        }
    }
    RS_LSTAMP(1);
    // ---- per-lane constants of the 6 lane bits: role mask, field shift, table offset
    uint32_t rm[6], sh[6], to[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t role = (lane >> j) & 1u;
        rm[j] = 0u - role;
        sh[j] = role << 2;
        to[j] = ((lane >> (j + 1)) << 4) + role * (2u * G::NT * 16u);
    }
    const uint32_t a1 = G::kA1Base + wave * G::kRegion, a3 = G::kA3Base + wave * G::kRegion;

    // phase-A IFFT region (written and read by this wave only: LDS ops of a wave are in order)
#pragma unroll
    for (int k = 0; k < K1; ++k) {
        const uint32_t q = lane + 64u * k;
        if (q < P * G::kA1) put(a1, q / P, q % P, v1[k]);
    }
    RS_LSTAMP(2);
    // the column: rows outside the caller's matrices are zero
    uint32_t v;
    {
        w[0] = okm & 1u ? w[0] : 0u;
        w[1] = okm & 2u ? w[1] : 0u;
        pair_xpose(w[0], w[1], lane);  // lane 2k: (lo, hi) of row 2k, lane 2k+1: of row 2k+1
        const uint32_t s = !io.bytes && (io.lo & 2u) ? 0x07060302u : 0x05040100u;
        v = io.bytes ? (w[0] & 0xFFFFu) | (w[1] << 16) : __builtin_amdgcn_perm(w[1], w[0], s);
    }

    // ---- the 2L layers; tables of layer k + 2 are read while layer k runs
    uint32_t tb[2][8];
    auto base_of = [&](auto kc) -> uint32_t {
        constexpr int k = decltype(kc)::value;
        constexpr int rg = Q::region(k);
        return rg == 0 ? a1 : rg == 1 ? G::kShIBase : rg == 2 ? G::kShFBase : a3;
    };
    auto request = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int J = Q::lane_bit(k);
        const uint8_t *p = lds8 + base_of(kc) + Q::slot0(k) * 16u + to[J];
        const uint4 x = *reinterpret_cast<const uint4 *>(p);
        const uint4 y = *reinterpret_cast<const uint4 *>(p + G::NT * 16u);
        tb[k & 1][0] = x.x, tb[k & 1][1] = x.y, tb[k & 1][2] = x.z, tb[k & 1][3] = x.w;
        tb[k & 1][4] = y.x, tb[k & 1][5] = y.y, tb[k & 1][6] = y.z, tb[k & 1][7] = y.w;
    };
    auto remap = [&](uint32_t from, uint32_t to_row) {
        __syncthreads();
        plane[lswz(from)] = v;
        __syncthreads();
        v = plane[lswz(to_row)];
    };
    const uint32_t row_a = tid, row_b = (lane << G::WB) | wave;
    auto step = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int J = Q::lane_bit(k);
        // region boundaries: the remaps (and the staging of the later regions)
        if constexpr (k == 6) {
#pragma unroll
            for (int i = 0; i < KS; ++i) {
                const uint32_t q = tid + n * i;
                if (q < kShP) {
                    const uint32_t t = q / P;
                    const uint32_t base = t < G::kShI ? G::kShIBase : G::kShFBase;
                    put(base, t < G::kShI ? t : t - G::kShI, q % P, vs[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < K3; ++i) {
                const uint32_t q = lane + 64u * i;
                if (q < P * G::kA3) put(a3, q / P, q % P, v3[i]);
            }
            RS_LSTAMP(4);
            remap(row_a, row_b);  // (its barriers also publish the shared tables)
            RS_LSTAMP(5);
            request(std::integral_constant<int, 6>{});
            request(std::integral_constant<int, 7>{});
        } else if constexpr (k == 2 * L - G::WB) {
            RS_LSTAMP(6);
            remap(row_b, row_a);
            RS_LSTAMP(7);
            request(std::integral_constant<int, k>{});
            if constexpr (k + 1 < 2 * L) request(std::integral_constant<int, k + 1>{});
        }
#ifndef RS_LANE_SKIP_LAYERS  // tools/lane_probe.hip ablation
        if constexpr (Q::bit(k) == L - 1 && RS_MONO_ZERO_TOP) {
            // skew offset 0 (image 0): the top layer's twiddle is zero (rs_mono.hip
            // run_seq zero_top), both butterflies reduce to b ^= a
            if ((Q::ifft(k) ? A.ifft_img : A.fft_img) == 0) v ^= partner<J>(v, rm[J]) & rm[J];
            else lane_layer<J, Q::ifft(k)>(v, tb[k & 1], rm[J], sh[J]);
        } else {
            lane_layer<J, Q::ifft(k)>(v, tb[k & 1], rm[J], sh[J]);
        }
#else
        v ^= tb[k & 1][0] ^ tb[k & 1][7];
#endif
        // the next request of this buffer, unless it lies past a remap
        constexpr int nk = k + 2;
        if constexpr (nk < 2 * L && nk != 6 && nk != 7 && nk != 2 * L - G::WB && nk != 2 * L - G::WB + 1)
            request(std::integral_constant<int, nk>{});
    };
    request(std::integral_constant<int, 0>{});
    request(std::integral_constant<int, 1>{});
    RS_LSTAMP(3);
    static_for<0, 2 * L>(step);
    RS_LSTAMP(8);

    // ---- stores (placement A), paired like the loads; only rows of A.dst
    uint32_t o[2] = {v & 0xFFFFu, v >> 16};
    pair_xpose(o[0], o[1], lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t r = (tid & ~1u) | uint32_t(j);
        if (r >= A.dst.row_begin && r < A.dst.row_end)
            st_half(dst + uint64_t(r - A.dst.row_begin) * A.dst.stride + off, o[j], io);
    }
    RS_LSTAMP(9);
}

}  // namespace

bool lane_supported(int L) { return L >= 8 && L <= 10; }

hipError_t launch_lane(int L, const MonoCore &A, hipStream_t s) {
    if (A.elems != 2 || A.chunks != 1) return hipErrorInvalidValue;
    auto go = [&](auto lc, auto bc) -> hipError_t {
        constexpr int LL = decltype(lc)::value;
        constexpr bool BATCH = decltype(bc)::value;
        using G = LaneGeo<LL>;
        static std::atomic<uint64_t> attr_devs{0};
        const void *fn = reinterpret_cast<const void *>(&k_lane<LL, BATCH>);
        hipError_t e = lds_attr_once(attr_devs, fn, int(G::kBytes));
        if (e != hipSuccess) return e;
        k_lane<LL, BATCH><<<dim3(8u * A.packs_per_xcd, BATCH ? A.stripes : 1), G::n, G::kBytes, s>>>(A);
        snprintf(launch_name_buf(), kLaunchNameBytes, "k_lane<%d, %s>", LL, BATCH ? "true" : "false");
        return hipGetLastError();
    };
    const bool batch = A.stripes > 1;
    switch (L) {
        case 8: return batch ? go(std::integral_constant<int, 8>{}, std::true_type{})
                             : go(std::integral_constant<int, 8>{}, std::false_type{});
        case 9: return batch ? go(std::integral_constant<int, 9>{}, std::true_type{})
                             : go(std::integral_constant<int, 9>{}, std::false_type{});
        case 10: return batch ? go(std::integral_constant<int, 10>{}, std::true_type{})
                              : go(std::integral_constant<int, 10>{}, std::false_type{});
        default: return hipErrorNotSupported;
    }
}

}  // namespace rs
