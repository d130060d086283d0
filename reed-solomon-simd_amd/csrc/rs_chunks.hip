// Multi-chunk column kernel ("k_chunks") of the MI355X Reed-Solomon engine:
// encodes whose transform has n = 2^L <= 128 rows and several chunks -- HighRate
// with N > n originals (src/rate/rate_high.rs:44-87: recovery = FFT_0(XOR_c
// IFFT_{c n + n}(chunk c)), e.g. 1000:100) and LowRate with M > n recovery rows
// (src/rate/rate_low.rs:44-87: recovery chunk c = FFT_{c n + n}(IFFT_0(original)),
// e.g. 128:1024) -- in one launch.
//
// One workgroup owns one pack (4 or 2 elements of every shard, reference block
// layout src/algorithm.md:18-31) as k_mono does (rs_mono.hip), but its waves
// split the CHUNKS: a whole n-row transform fits one wave (2 rows per lane, row
// bit 0 and the lane bits; every layer in registers, DPP / permlane
// transposes, no barrier), so wave w transforms chunks w, w + W, ... at once
// with the other waves.  HighRate XOR-folds the waves' IFFT results through LDS
// and wave 0 runs the FFT; LowRate runs the IFFT in every wave (the same
// inputs, no barrier) and wave w the FFTs of output chunks w, w + W, ....
// (The chunk-serial forms -- one workgroup transforming the chunks one after
// another, or one launch per step with the chunks over the grid -- take
// 13-30 us for 1000:100 x 1 KiB, profiles/r05g.)
//
// Twiddles: each wave stages its chunk's layer-ordered image (the layout of
// k_mono's images, rs_codec.cpp mono_images: table of layer b, group g at slot
// n - n / 2^b + g) into a wave-private LDS region of 20-word slots (16 lanes'
// ds_read_b128 of 16 different slots then hit 16 different bank groups).  The
// images hold 8-word basis tables (rs_codec.cpp basis_images), expanded while
// staging (CTabsBasis, CTabsBasis4).
//
// Placement of a wave's n rows: lane l, register k.  Before IFFT layer b the
// register bit holds row bit b, lane bits j < b row bits j, lane bits j >= b row
// bits j + 1 (a 2x2 register / lane-bit transpose, xpose<b - 1>, moves the
// register bit up one layer); the group of the lane's pair at layer b is
// lane >> b.  The FFT walks the same placements backwards.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <type_traits>

#include "rs_device.hpp"
#include "rs_gf.hpp"

namespace rs {
namespace {

// 2x2 transpose of (register pair, lane bit J) -- as rs_mono.hip xpose: the lane
// with bit J clear ends with (a, partner's a), its partner with (a-lane's b, b)
template <int J>
__device__ __forceinline__ void cx(uint32_t &a, uint32_t &b, uint32_t lane) {
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

#ifdef RS_CHUNK_STAMPS  // tools/chunks_probe.hip: per-workgroup timestamps of wave 0 and the last wave
__device__ uint64_t g_chunk_stamps[4096][2][8];
#define RS_CSTAMP(i)                                                                                        \
    do {                                                                                                    \
        asm volatile("" ::: "memory");                                                                      \
        if ((threadIdx.x & 63u) == 0 && (threadIdx.x == 0 || threadIdx.x == blockDim.x - 64) && blockIdx.x < 4096) \
            g_chunk_stamps[blockIdx.x][threadIdx.x ? 1 : 0][i] = __builtin_amdgcn_s_memrealtime();          \
    } while (0)
#else
#define RS_CSTAMP(i)
#endif

constexpr uint32_t kSlot = 20;  // LDS words per table slot
constexpr uint32_t kMaxWaves = 8;

template <int L, int E>
struct ChunkGeo {
    static_assert(L >= 2 && L <= 7, "k_chunks: transforms of 4 .. 128 rows (one wave, 2 rows per lane)");
    static constexpr uint32_t n = 1u << L;
    static constexpr uint32_t TW = E == 4 ? 20 : 16;     // table words (kPermWords / kPerm2Words)
    static constexpr uint32_t PC = TW / 4;               // 16-byte pieces per table
    static constexpr uint32_t region = (n - 1) * kSlot;  // LDS words of a wave's tables
    static constexpr uint32_t pieces = (n - 1) * PC;
    static constexpr int KP = int((pieces + 63) / 64);   // pieces per lane
    static constexpr uint32_t WPR = E == 4 ? 2 : 1;      // words per row
    static constexpr uint32_t plane = 64 * 2 * WPR;      // LDS words of a wave's folded rows, per pack
    static constexpr size_t bytes(uint32_t waves, bool high, int pw) {
        return size_t(waves) * (region + (high ? plane * pw : 0)) * 4;
    }
};

// A wave's rows: register k of lane l (words lo, and hi for 4-element packs) of
// each of the wave's PW packs (the tables, pack-independent, serve all of them)
template <int PW>
struct CRows {
    uint32_t lo[PW][2], hi[PW][2];
};

// 2-element tables built in the kernel from their basis images (rs_codec.cpp
// basis_images): per table the 16 products P(e_i) = x * e_i of the multiplier with
// the Cantor basis elements, 8 words (word 2f = P(e_2f) | P(e_2f+1) << 16 for the
// low byte's 2-bit field f, word 2f + 1 the high byte's) -- half the bytes of the
// 16-word table.  Multiplication by a constant is GF(2)-linear, so field f's four
// lookups are {0, a, b, a ^ b} (a, b its two basis products): a word X = a | b << 16
// gives the table words [0, a_lo, b_lo, (a ^ b)_lo] and [0, a_hi, b_hi, (a ^ b)_hi]
// (gf_tables.cpp fill_perm2) by two v_perm_b32 each.  1000:100 x 1 KiB 10.8 -> 5.9 us
// per launch against staging the 16-word images (profiles/r05g/chunks_basis.txt):
// the staging's L2 requests, not the 32 VALU per table, bound the launch.
template <int L>
struct CTabsBasis {
    static constexpr uint32_t n = 1u << L, tabs = n - 1;
    static constexpr int KT = int((tabs + 63) / 64);  // tables per lane
    uint4 v[KT][2];
    __device__ __forceinline__ void issue(const uint32_t *img, uint32_t lane) {
        const uint4 *src = reinterpret_cast<const uint4 *>(img);
        static_for<0, KT>([&](auto kc) {
            const uint32_t t = lane + 64u * decltype(kc)::value, tt = t < tabs ? t : tabs - 1;
            v[kc][0] = src[2 * tt];
            v[kc][1] = src[2 * tt + 1];
        });
    }
    __device__ __forceinline__ void write(uint32_t *region, uint32_t lane) const {
        static_for<0, KT>([&](auto kc) {
            const uint32_t t = lane + 64u * decltype(kc)::value;
            if (t < tabs) {
                const uint32_t X[8] = {v[kc][0].x, v[kc][0].y, v[kc][0].z, v[kc][0].w,
                                       v[kc][1].x, v[kc][1].y, v[kc][1].z, v[kc][1].w};
                uint32_t w[16];
                static_for<0, 4>([&](auto fc) {
                    constexpr int f = decltype(fc)::value;
                    const uint32_t A = X[2 * f], C = X[2 * f + 1];
                    const uint32_t tA = A ^ __builtin_amdgcn_alignbit(A, A, 16), tC = C ^ __builtin_amdgcn_alignbit(C, C, 16);
                    w[4 * f + 0] = __builtin_amdgcn_perm(tA, A, 0x0402000Cu);  // direct: low-byte field, low bytes
                    w[4 * f + 1] = __builtin_amdgcn_perm(tC, C, 0x0503010Cu);  // direct: high-byte field, high bytes
                    w[4 * f + 2] = __builtin_amdgcn_perm(tC, C, 0x0402000Cu);  // cross: high-byte field, low bytes
                    w[4 * f + 3] = __builtin_amdgcn_perm(tA, A, 0x0503010Cu);  // cross: low-byte field, high bytes
                });
                uint4 *d = reinterpret_cast<uint4 *>(region) + t * (kSlot / 4);
                static_for<0, 4>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    d[q] = uint4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
                });
            }
        });
    }
};

// 4-element tables (gf_tables.cpp fill_perm: 5 words per input byte B and output
// byte O, 3-bit fields) from 8 basis words: per input byte B, word 4B = P0 | P1 << 16,
// 4B + 1 = P3 | P4 << 16, 4B + 2 = P6 | P7 << 16, 4B + 3 = P2 | P5 << 16 (Pj = x * e_8B+j).
// Field bits 0-2: entries [0, P0, P1, P0^P1] then the same XOR P2 (byte O of each);
// bits 3-5 likewise with P3, P4, P5; bits 6-7: [0, P6, P7, P6^P7].  ~44 VALU per
// table for 32 of its 80 bytes.
template <int L>
struct CTabsBasis4 {
    static constexpr uint32_t n = 1u << L, tabs = n - 1;
    static constexpr int KT = int((tabs + 63) / 64);
    uint4 v[KT][2];
    __device__ __forceinline__ void issue(const uint32_t *img, uint32_t lane) {
        const uint4 *src = reinterpret_cast<const uint4 *>(img);
        static_for<0, KT>([&](auto kc) {
            const uint32_t t = lane + 64u * decltype(kc)::value, tt = t < tabs ? t : tabs - 1;
            v[kc][0] = src[2 * tt];
            v[kc][1] = src[2 * tt + 1];
        });
    }
    __device__ __forceinline__ void write(uint32_t *region, uint32_t lane) const {
        static_for<0, KT>([&](auto kc) {
            const uint32_t t = lane + 64u * decltype(kc)::value;
            if (t < tabs) {
                uint4 o[5];
                basis4_expand(v[kc][0], v[kc][1], o);
                uint4 *d = reinterpret_cast<uint4 *>(region) + t * (kSlot / 4);
                static_for<0, 5>([&](auto qc) { d[decltype(qc)::value] = o[decltype(qc)::value]; });
            }
        });
    }
};

template <int L, int E, int B>
__device__ __forceinline__ void c_table(const uint32_t *region, uint32_t lane, uint32_t (&t)[ChunkGeo<L, E>::TW]) {
    using G = ChunkGeo<L, E>;
    constexpr uint32_t groups = G::n >> (B + 1), base = G::n - (G::n >> B);
    const uint32_t slot = base + ((lane >> B) & (groups - 1u));
    const uint4 *p = reinterpret_cast<const uint4 *>(region + slot * kSlot);
    static_for<0, int(G::PC)>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const uint4 x = p[q];
        t[4 * q] = x.x, t[4 * q + 1] = x.y, t[4 * q + 2] = x.z, t[4 * q + 3] = x.w;
    });
}

template <int J, int E, int PW>
__device__ __forceinline__ void c_xpose(CRows<PW> &r, uint32_t lane) {
    static_for<0, PW>([&](auto pc) {
        cx<J>(r.lo[pc][0], r.lo[pc][1], lane);
        if constexpr (E == 4) cx<J>(r.hi[pc][0], r.hi[pc][1], lane);
    });
}

// Top layer of a transform with skew offset 0 (zero twiddle, rs_mono.hip
// run_seq zero_top): both butterflies reduce to b ^= a.
template <int E, int PW>
__device__ __forceinline__ void c_xor_layer(CRows<PW> &r) {
    static_for<0, PW>([&](auto pc) {
        r.lo[pc][1] ^= r.lo[pc][0];
        if constexpr (E == 4) r.hi[pc][1] ^= r.hi[pc][0];
    });
}

// IFFT layers 0..L-1 (engine_naive.rs:75-105), placement as in the header;
// zero_top: skew offset 0
template <int L, int E, int PW>
__device__ __forceinline__ void c_ifft(CRows<PW> &r, const uint32_t *region, uint32_t lane, bool zero_top = false) {
    static_for<0, L>([&](auto bc) {
        constexpr int B = decltype(bc)::value;
        if constexpr (B > 0) c_xpose<B - 1, E>(r, lane);
        if constexpr (B == L - 1 && RS_MONO_ZERO_TOP) {
            if (zero_top) {
                c_xor_layer<E>(r);
                return;
            }
        }
        uint32_t t[ChunkGeo<L, E>::TW];
        c_table<L, E, B>(region, lane, t);
        static_for<0, PW>([&](auto pc) {
            if constexpr (E == 2) ifft_bfly2(r.lo[pc][0], r.lo[pc][1], t);
            else ifft_bfly(r.lo[pc][0], r.hi[pc][0], r.lo[pc][1], r.hi[pc][1], t);
        });
    });
}

// FFT layers L-1..0 (engine_naive.rs:43-73)
template <int L, int E, int PW>
__device__ __forceinline__ void c_fft(CRows<PW> &r, const uint32_t *region, uint32_t lane, bool zero_top = false) {
    static_for<0, L>([&](auto ic) {
        constexpr int B = L - 1 - decltype(ic)::value;
        if constexpr (B < L - 1) c_xpose<B, E>(r, lane);
        if constexpr (B == L - 1 && RS_MONO_ZERO_TOP) {
            if (zero_top) {
                c_xor_layer<E>(r);
                return;
            }
        }
        uint32_t t[ChunkGeo<L, E>::TW];
        c_table<L, E, B>(region, lane, t);
        static_for<0, PW>([&](auto pc) {
            if constexpr (E == 2) fft_bfly2(r.lo[pc][0], r.lo[pc][1], t);
            else fft_bfly(r.lo[pc][0], r.hi[pc][0], r.lo[pc][1], r.hi[pc][1], t);
        });
    });
}

// The wave's rows of chunk c in the starting placement (row (lane << 1) | k).
// Lanes 2m and 2m + 1 hold rows 4m .. 4m + 3 between them, and they load (and
// store) those rows as pairs: step j, the even lane the low half, the odd lane
// the high half of row 4m + j (one 64-byte block) -- 32 rows per wave
// instruction instead of 64, the row I/O being bound by blocks per instruction
//  -- and swap the halves they do not keep (DPP).
template <int E>
__device__ __forceinline__ uint32_t c_half(const RowMap &m, uint32_t row, const PackIO &io, bool high_half) {
    if (row < m.row_begin || row >= m.row_end) return 0;
    const uint8_t *p = m.base + uint64_t(row - m.row_begin) * m.stride + io.lo + (high_half ? io.hi_delta : 0u);
    if constexpr (E == 4) return ld_word(p, io);
    else return ld_half(p, io);
}
template <int E>
__device__ __forceinline__ void c_put_half(const RowMap &m, uint32_t row, const PackIO &io, bool high_half, uint32_t v) {
    if (row < m.row_begin || row >= m.row_end) return;
    uint8_t *p = const_cast<uint8_t *>(m.base) + uint64_t(row - m.row_begin) * m.stride + io.lo +
                 (high_half ? io.hi_delta : 0u);
    if constexpr (E == 4) st_word(p, v, io);
    else st_half(p, v, io);
}
template <int L, int E>
__device__ __forceinline__ void c_load_pack(const RowMap &m, uint32_t c, const PackIO &io, uint32_t lane,
                                            uint32_t (&rlo)[2], uint32_t (&rhi)[2]) {
    constexpr uint32_t n = 1u << L;
    const bool odd = lane & 1u;
    const uint32_t local0 = (lane & ~1u) << 1;
    uint32_t v[4];
    static_for<0, 4>([&](auto jc) {
        constexpr uint32_t j = decltype(jc)::value;
#ifndef RS_CHUNK_SKIP_ROWS  // (tools/chunks_probe.hip ablation)
        v[j] = local0 + j < n ? c_half<E>(m, c * n + local0 + j, io, odd) : 0u;
#else
        v[j] = (c * n + local0 + j) * 0x9E3779B9u + lane;
#endif
    });
    // even lane: keeps the low halves of rows 0, 1, gets their high halves; odd: rows 2, 3
    const uint32_t g0 = xor_lane<0>(odd ? v[0] : v[2]), g1 = xor_lane<0>(odd ? v[1] : v[3]);
    const uint32_t lo0 = odd ? g0 : v[0], lo1 = odd ? g1 : v[1];
    const uint32_t hi0 = odd ? v[2] : g0, hi1 = odd ? v[3] : g1;
    if constexpr (E == 4) {
        rlo[0] = lo0, rlo[1] = lo1, rhi[0] = hi0, rhi[1] = hi1;
    } else {
        rlo[0] = lo0 | (hi0 << 16), rlo[1] = lo1 | (hi1 << 16);
        rhi[0] = rhi[1] = 0;
    }
}
template <int L, int E>
__device__ __forceinline__ void c_store_pack(const RowMap &m, uint32_t c, const PackIO &io, uint32_t lane,
                                             const uint32_t (&rlo)[2], const uint32_t (&rhi)[2]) {
    constexpr uint32_t n = 1u << L;
    const bool odd = lane & 1u;
    const uint32_t local0 = (lane & ~1u) << 1;
    uint32_t lo[2], hi[2];
    static_for<0, 2>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        lo[k] = E == 4 ? rlo[k] : rlo[k] & 0xFFFFu;
        hi[k] = E == 4 ? rhi[k] : rlo[k] >> 16;
    });
    // even lane stores the low halves of rows 0..3, odd the high halves
    const uint32_t g0 = xor_lane<0>(odd ? lo[0] : hi[0]), g1 = xor_lane<0>(odd ? lo[1] : hi[1]);
    const uint32_t w[4] = {odd ? g0 : lo[0], odd ? g1 : lo[1], odd ? hi[0] : g0, odd ? hi[1] : g1};
    static_for<0, 4>([&](auto jc) {
        constexpr uint32_t j = decltype(jc)::value;
        if (local0 + j < n) c_put_half<E>(m, c * n + local0 + j, io, odd, w[j]);
    });
}

// A wave's PW packs (pk[p] >= A.packs: none; zero rows, nothing stored)
template <int L, int E, int PW>
__device__ __forceinline__ void c_load_chunk(const RowMap &m, uint32_t c, const PackIO (&io)[PW], const bool (&ok)[PW],
                                             uint32_t lane, CRows<PW> &r) {
    static_for<0, PW>([&](auto pc) {
        if (ok[pc]) c_load_pack<L, E>(m, c, io[pc], lane, r.lo[pc], r.hi[pc]);
        else r.lo[pc][0] = r.lo[pc][1] = r.hi[pc][0] = r.hi[pc][1] = 0;
    });
}
template <int L, int E, int PW>
__device__ __forceinline__ void c_store_chunk(const RowMap &m, uint32_t c, const PackIO (&io)[PW], const bool (&ok)[PW],
                                              uint32_t lane, const CRows<PW> &r) {
    static_for<0, PW>([&](auto pc) {
        if (ok[pc]) c_store_pack<L, E>(m, c, io[pc], lane, r.lo[pc], r.hi[pc]);
    });
}

template <int L, int E, bool HIGH, int PW>
__global__ void __launch_bounds__(64 * kMaxWaves) k_chunks(const MonoCore A) {
    using G = ChunkGeo<L, E>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t b = blockIdx.x;
    // pack group (XCD-aware, as k_mono; packs_per_xcd counts groups of PW packs here)
    const uint32_t pg = (b & 7u) * A.packs_per_xcd + (b >> 3);
    if (pg * PW >= A.packs) return;
    PackIO io[PW];
    bool ok[PW];
    static_for<0, PW>([&](auto pc) {
        const uint32_t pk = pg * PW + uint32_t(decltype(pc)::value);
        ok[pc] = pk < A.packs;
        io[pc] = E == 4 ? pack_io(A.fmt, ok[pc] ? pk : pg * PW) : pack_io2(A.fmt, ok[pc] ? pk : pg * PW);
    });
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t W = blockDim.x >> 6;
    uint32_t *region = lds + wave * G::region;
    std::conditional_t<E == 2, CTabsBasis<L>, CTabsBasis4<L>> tabs;  // basis images, both formats
    RS_CSTAMP(0);
    const uint32_t *img_base = A.img;
    if constexpr (HIGH) {
        // chunk c: IFFT with skew offset c n + n (image ifft_img + c), XOR-folded
        CRows<PW> acc;
        static_for<0, PW>([&](auto pc) { acc.lo[pc][0] = acc.lo[pc][1] = acc.hi[pc][0] = acc.hi[pc][1] = 0; });
        // software-pipelined: chunk c + W's rows and image pieces are requested
        // before chunk c's layers run
        CRows<PW> r;
        uint32_t c = wave;
        c_load_chunk<L, E>(A.src[0], c, io, ok, lane, r);
        tabs.issue(img_base + uint64_t(A.ifft_img + c * A.ifft_img_step) * A.img_words, lane);
        while (c < A.chunks) {
            tabs.write(region, lane);
            RS_CSTAMP(1);
            CRows<PW> cur = r;
            const uint32_t nc = c + W;
            if (nc < A.chunks) {
                c_load_chunk<L, E>(A.src[0], nc, io, ok, lane, r);
                tabs.issue(img_base + uint64_t(A.ifft_img + nc * A.ifft_img_step) * A.img_words, lane);
            }
            c_ifft<L, E>(cur, region, lane);
            static_for<0, PW>([&](auto pc) {
                static_for<0, 2>([&](auto kc) {
                    acc.lo[pc][kc] ^= cur.lo[pc][kc];
                    acc.hi[pc][kc] ^= cur.hi[pc][kc];
                });
            });
            RS_CSTAMP(2);
            c = nc;
        }
        RS_CSTAMP(3);
        uint32_t *plane = lds + W * G::region;
        // plane word of (wave w, pack p, register k, word h): ((h * PW + p) * W + w) * 2 + k, times 64 lanes
        auto at = [&](uint32_t w, int p, int k, int h) { return ((((h * PW + p) * W + w) * 2) + k) * 64 + lane; };
        if (wave != 0) {
            static_for<0, PW>([&](auto pc) {
                static_for<0, 2>([&](auto kc) {
                    plane[at(wave, pc, kc, 0)] = acc.lo[pc][kc];
                    if constexpr (E == 4) plane[at(wave, pc, kc, 1)] = acc.hi[pc][kc];
                });
            });
        } else {
            tabs.issue(img_base + uint64_t(A.fft_img) * A.img_words, lane);  // the FFT's (skew offset 0)
        }
        __syncthreads();
        RS_CSTAMP(4);
        if (wave != 0) return;
        for (uint32_t w = 1; w < W; ++w)
            static_for<0, PW>([&](auto pc) {
                static_for<0, 2>([&](auto kc) {
                    acc.lo[pc][kc] ^= plane[at(w, pc, kc, 0)];
                    if constexpr (E == 4) acc.hi[pc][kc] ^= plane[at(w, pc, kc, 1)];
                });
            });
        tabs.write(region, lane);
        c_fft<L, E>(acc, region, lane, A.fft_img == 0);
        RS_CSTAMP(5);
        c_store_chunk<L, E>(A.dst, 0, io, ok, lane, acc);
        RS_CSTAMP(6);
    } else {
        // IFFT of the originals (skew offset 0) in every wave, then output chunk c
        // FFT'd with skew offset c n + n (image fft_img + c)
        CRows<PW> x;
        c_load_chunk<L, E>(A.src[0], 0, io, ok, lane, x);
        tabs.issue(img_base + uint64_t(A.ifft_img) * A.img_words, lane);
        tabs.write(region, lane);
        uint32_t c = wave;
        tabs.issue(img_base + uint64_t(A.fft_img + c * A.fft_img_step) * A.img_words, lane);  // in flight during the IFFT
        RS_CSTAMP(1);
        c_ifft<L, E>(x, region, lane, A.ifft_img == 0);
        RS_CSTAMP(2);
        while (c < A.chunks) {
            tabs.write(region, lane);
            RS_CSTAMP(3);
            const uint32_t nc = c + W;
            if (nc < A.chunks) tabs.issue(img_base + uint64_t(A.fft_img + nc * A.fft_img_step) * A.img_words, lane);
            CRows<PW> y = x;
            c_fft<L, E>(y, region, lane);
            RS_CSTAMP(5);
            c_store_chunk<L, E>(A.dst, c, io, ok, lane, y);
            RS_CSTAMP(6);
            c = nc;
        }
    }
}

}  // namespace

bool chunks_supported(int L) { return L >= 2 && L <= 7; }

hipError_t launch_chunks(int L, bool high, const MonoCore &A, hipStream_t s, int pw) {
    if (A.packs == 0) return hipSuccess;
    if (A.chunks < 2 || A.stripes != 1 || (A.elems != 2 && A.elems != 4) || A.nsrc != 1) return hipErrorInvalidValue;
    if (pw != 1 && pw != 2 && pw != 4) return hipErrorInvalidValue;
    const uint32_t waves = A.chunks < kMaxWaves ? A.chunks : kMaxWaves;
    MonoCore B = A;
    B.packs_per_xcd = ((A.packs + pw - 1) / pw + 7) / 8;  // pack groups per XCD
    auto go = [&](auto lc, auto ec, auto hc, auto pc) -> hipError_t {
        constexpr int LL = decltype(lc)::value, E = decltype(ec)::value, PW = decltype(pc)::value;
        constexpr bool H = decltype(hc)::value;
        using G = ChunkGeo<LL, E>;
        const size_t lds = G::bytes(waves, H, PW);
        static std::atomic<uint64_t> attr_devs{0};
        const void *fn = reinterpret_cast<const void *>(&k_chunks<LL, E, H, PW>);
        hipError_t e = lds_attr_once(attr_devs, fn, int(G::bytes(kMaxWaves, H, PW)));
        if (e != hipSuccess) return e;
        k_chunks<LL, E, H, PW><<<8u * B.packs_per_xcd, 64u * waves, lds, s>>>(B);
        snprintf(launch_name_buf(), kLaunchNameBytes, "k_chunks<%d, %d, %s, %d>", LL, E, H ? "true" : "false", PW);
        return hipGetLastError();
    };
    auto by_pw = [&](auto lc, auto ec, auto hc) -> hipError_t {
        if (pw == 1) return go(lc, ec, hc, std::integral_constant<int, 1>{});
        if (pw == 2) return go(lc, ec, hc, std::integral_constant<int, 2>{});
        return go(lc, ec, hc, std::integral_constant<int, 4>{});
    };
    auto by_e = [&](auto lc) -> hipError_t {
        if (A.elems == 2) return high ? by_pw(lc, std::integral_constant<int, 2>{}, std::true_type{})
                                      : by_pw(lc, std::integral_constant<int, 2>{}, std::false_type{});
        return high ? by_pw(lc, std::integral_constant<int, 4>{}, std::true_type{})
                    : by_pw(lc, std::integral_constant<int, 4>{}, std::false_type{});
    };
    switch (L) {
        case 2: return by_e(std::integral_constant<int, 2>{});
        case 3: return by_e(std::integral_constant<int, 3>{});
        case 4: return by_e(std::integral_constant<int, 4>{});
        case 5: return by_e(std::integral_constant<int, 5>{});
        case 6: return by_e(std::integral_constant<int, 6>{});
        case 7: return by_e(std::integral_constant<int, 7>{});
        default: return hipErrorNotSupported;
    }
}

}  // namespace rs
