// HIP kernels of the MI355X (gfx950) Reed-Solomon GF(2^16) engine.
//
// The hot path is the additive FFT / IFFT of the Leopard construction over the
// shard matrix (reference: src/engine/engine_naive.rs:43-105 semantics,
// src/rate/rate_high.rs / rate_low.rs call sites).  Every engine op acts
// independently on each element column, so a transform over n rows is split
// into passes over row SETS x 64-pack column SLICES.
//
// GF multiply: multiplication by a constant is GF(2)-linear, so x*m is the XOR
// of table lookups on 3-bit fields of x.  Four elements are packed as one
// 32-bit word of low bytes + one of high bytes (the reference's block layout),
// and v_perm_b32 performs 4 byte lookups into an 8-entry table at once
// (12 v_perm + 10 field extracts + 6 v_bitop3 XOR3 per 4 elements).
// Lanes run along the columns (packs) of the shard matrix; the twiddle tables
// of a pass are staged in LDS once per workgroup.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>

#include "rs_device.hpp"
#include "rs_gf.hpp"

namespace rs {
namespace {


// Block pruning of the decode's fused top pass (PassArgs::bfly_prune; 0: the
// variant without it, for A/B)
#ifndef RS_PASS_BFLY_PRUNE
#define RS_PASS_BFLY_PRUNE 1
#endif

// -------------------------------------------------------------------------
// Pass kernel.
//   K   : log2 rows per set (the butterfly layers this pass runs)
//   LR  : log2 rows a lane holds in registers
//   SPL : log2 packs per workgroup column slice
// A workgroup is G = 2^(K-LR) row groups x SP packs: thread t works on pack
// t % SP of row group g = t / SP.  The K local row bits are covered by
// register PHASES: in phase p a lane's registers run over local row bits
// [s_p, s_p + LR), s_p = min(p*LR, K-LR), the remaining bits come from g.
// Layer b runs in phase min(b / LR, NPH - 1); a phase change is an exchange
// of the rows through LDS.  Small slices (SPL < 6) spread a small shard matrix
// over more workgroups; then g differs inside a wave and row addresses and
// twiddle tables are per lane instead of wave-uniform.
template <int K, int LR, int SPL>
struct Pass {
    static constexpr int R = 1 << LR;
    static constexpr int SP = 1 << SPL;
    static constexpr int G = 1 << (K - LR);
    static constexpr int kThreads = SP * G;
    static constexpr int NPH = K == 0 ? 1 : (K + LR - 1) / LR;
    static constexpr bool kUniform = SPL >= 6;
    // Left alone, the compiler interleaves every butterfly of a layer and
    // hoists all their tables: with 8 rows per lane that costs occupancy or
    // spills, so wide shapes run one table / butterfly at a time per wave.
    static constexpr bool kSerial = R >= 8;
    static_assert(K == 0 || (LR >= 1 && LR <= K), "register bits must fit the set");
    static_assert(kThreads >= 64, "at least one full wave");

    static constexpr int start(int p) { return p * LR < K - LR ? p * LR : K - LR; }
    static constexpr int phase_of(int b) { return LR == 0 || b / (LR ? LR : 1) >= NPH - 1 ? NPH - 1 : b / (LR ? LR : 1); }

    // local row held in register i in phase PH ('+': disjoint bits, lets the
    // register index fold into immediate offsets)
    template <int PH>
    static __device__ __forceinline__ uint32_t lrow(uint32_t g, int i) {
        if constexpr (G == 1) {
            return uint32_t(i);
        } else {
            constexpr int s = start(PH);
            const uint32_t lo = g & ((1u << s) - 1u), hi = g >> s;
            return lo + (uint32_t(i) << s) + (hi << (s + LR));
        }
    }
};

struct Ctx {
    uint32_t g, p, s_lo, s_hi, a, pk_off;  // pk_off: the pack's low word in a row (work buffers: high word + 32)
    bool pk_ok;
    PackIO io;  // the pack in the caller's src / dst rows (tail shards, unaligned matrices)
    __device__ __forceinline__ uint32_t grow(uint32_t j, int K) const { return s_lo + (j << a) + (s_hi << (a + K)); }
};

// Keep a row index's address math at its use (not hoisted, which costs
// registers); wave-uniform indices stay scalar.
template <bool UNIFORM>
__device__ __forceinline__ uint32_t pin(uint32_t r) {
    if constexpr (UNIFORM) {
        r = __builtin_amdgcn_readfirstlane(r);
        asm volatile("" : "+s"(r));
    } else {
        asm volatile("" : "+v"(r));
    }
    return r;
}

// Row words of the work buffers.
__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) { *reinterpret_cast<uint32_t *>(p) = v; }

// LDS layout (dynamic, 16-byte aligned), in 32-bit words:
//   planes : 2 x (2^K rows x SP packs): low and high words of the exchange
//   tabI   : 2^K - 1 twiddle tables (20 words) of the IFFT in flight
//   tabF   : same for the FFT          (slot = 2^K - 2^(K-b) + group, b = local layer)
//   tabS   : per-row scale tables of a decode load   (log factor f)
//   tabV   : per-row tables of a decode reveal       (log factor 65535 - f)
//   rinfo  : decode row info of the set's rows
template <int K, int SPL, int FLAGS>
struct Lds {
    static constexpr uint32_t kPlane = uint32_t(1u << SPL) << K;
    static constexpr uint32_t kTab = 20u << K;
    static constexpr bool I = FLAGS & kIfft, F = FLAGS & kFft, S = FLAGS & kScale, V = FLAGS & kReveal;
    static constexpr uint32_t oI = 2 * kPlane;
    static constexpr uint32_t oF = oI + (I ? kTab : 0);
    static constexpr uint32_t oS = oF + (F ? kTab : 0);
    static constexpr uint32_t oV = oS + (S ? kTab : 0);
    static constexpr uint32_t oR = oV + (V ? kTab : 0);
    static constexpr uint32_t words = oR + ((S || V) ? (1u << K) : 0);
    static constexpr size_t bytes() { return size_t(words) * 4; }
};

// slot of the twiddle table of local layer b for local row j (bit b of j clear)
template <int K>
__device__ __forceinline__ uint32_t tw_slot(int b, uint32_t j) {
    return (1u << K) - (1u << (K - b)) + (j >> (b + 1));
}

// 16-byte piece t (of 5 per table) of the set's twiddle tables of a
// transform with skew offset delta.
template <int K>
__device__ __forceinline__ uint4 twiddle_piece(const PassArgs &A, const Ctx &c, uint32_t delta, uint32_t t) {
    const uint32_t slot = t / 5, piece = t - slot * 5;
    const uint32_t y = (1u << K) - slot;            // in [2, 2^K]
    const int b = K - (32 - __builtin_clz(y - 1));  // K - ceil(log2 y)
    const uint32_t grp = slot - ((1u << K) - (1u << (K - b)));
    const uint32_t row = c.grow(grp << (b + 1), K);
    const uint32_t gb = c.a + b;
    const uint32_t idx = (row & ~((2u << gb) - 1u)) + (1u << gb) + delta - 1u;
    return reinterpret_cast<const uint4 *>(A.tw)[idx * 5u + piece];
}

// Staging of a block's tables into LDS (null destinations are skipped), in
// two halves so several blocks' staging can share one memory round trip:
// load() issues every global load into registers, store() writes LDS.  NT =
// workgroup size.  Twiddles: one round trip; decode row tables: two (their
// address depends on the row's log factor).  No barrier.
// Basis tables (PassArgs::tab_basis): 2 pieces per table instead of 5, one table
// per thread, built into its 5 LDS pieces by basis4_expand (rs_gf.hpp).
template <int K>
__device__ __forceinline__ uint32_t twiddle_index(const Ctx &c, uint32_t delta, uint32_t slot) {
    const uint32_t y = (1u << K) - slot;            // in [2, 2^K]
    const int b = K - (32 - __builtin_clz(y - 1));  // K - ceil(log2 y)
    const uint32_t grp = slot - ((1u << K) - (1u << (K - b)));
    const uint32_t row = c.grow(grp << (b + 1), K);
    const uint32_t gb = c.a + b;
    return (row & ~((2u << gb) - 1u)) + (1u << gb) + delta - 1u;
}
template <int K, int NT>
struct BasisStager {
    static constexpr uint32_t kTw = (1u << K) - 1, kRw = 1u << K;  // tables
    static constexpr int PT = kTw ? (kTw + NT - 1) / NT : 1, PR = (kRw + NT - 1) / NT;
    uint4 vi[PT][2], vf[PT][2], vs[PR][2], vv[PR][2];
    uint32_t ri = 0;
    template <typename ST>
    __device__ __forceinline__ void load(const ST &st, const PassArgs &A, const Ctx &c, uint32_t chunk) {
        const uint32_t tid = threadIdx.x;
        const uint32_t dI = A.ifft_delta + chunk * A.ifft_delta_step, dF = A.fft_delta + chunk * A.fft_delta_step;
        const uint4 *tw = reinterpret_cast<const uint4 *>(A.tw);
        if (st.tabI || st.tabF) {
#pragma unroll
            for (int k = 0; k < PT; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kTw) {
                    if (st.tabI) {
                        const uint32_t i = twiddle_index<K>(c, dI, t);
                        vi[k][0] = tw[2 * i], vi[k][1] = tw[2 * i + 1];
                    }
                    if (st.tabF) {
                        const uint32_t i = twiddle_index<K>(c, dF, t);
                        vf[k][0] = tw[2 * i], vf[k][1] = tw[2 * i + 1];
                    }
                }
            }
        }
        if (st.tabS || st.tabV) {
            uint32_t f[PR];
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kRw) f[k] = st.ri_lds ? st.ri_lds[t] : A.rowinfo[c.grow(t, K) + chunk * A.n];
            }
            if (tid < (1u << K) && !st.ri_lds) ri = A.rowinfo[c.grow(tid, K) + chunk * A.n];
            const uint4 *lut = reinterpret_cast<const uint4 *>(A.lut);
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kRw) {
                    const uint32_t lf = f[k] & 0xFFFFu;
                    if (st.tabS) vs[k][0] = lut[2 * lf], vs[k][1] = lut[2 * lf + 1];
                    if (st.tabV) vv[k][0] = lut[2 * (65535u - lf)], vv[k][1] = lut[2 * (65535u - lf) + 1];
                }
            }
        }
    }
    template <typename ST>
    __device__ __forceinline__ void store(const ST &st) const {
        const uint32_t tid = threadIdx.x;
        auto put = [](uint32_t *tab, uint32_t t, const uint4 (&v)[2]) {
            uint4 o[5];
            basis4_expand(v[0], v[1], o);
#pragma unroll
            for (int q = 0; q < 5; ++q) reinterpret_cast<uint4 *>(tab)[t * 5 + q] = o[q];
        };
        if (st.tabI || st.tabF) {
#pragma unroll
            for (int k = 0; k < PT; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kTw) {
                    if (st.tabI) put(st.tabI, t, vi[k]);
                    if (st.tabF) put(st.tabF, t, vf[k]);
                }
            }
        }
        if (st.tabS || st.tabV) {
            if (tid < (1u << K) && !st.ri_lds) st.rinfo[tid] = ri;
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kRw) {
                    if (st.tabS) put(st.tabS, t, vs[k]);
                    if (st.tabV) put(st.tabV, t, vv[k]);
                }
            }
        }
    }
};

template <int K, int NT>
struct Stager {
    // in 16-byte pieces: 5 per 20-word table
    static constexpr uint32_t kTw = ((1u << K) - 1) * 5, kRw = 5u << K;
    static constexpr int PT = kTw ? (kTw + NT - 1) / NT : 1, PR = (kRw + NT - 1) / NT;
    uint32_t *tabI = nullptr, *tabF = nullptr, *tabS = nullptr, *tabV = nullptr, *rinfo = nullptr;
    const uint32_t *ri_lds = nullptr;  // row info already in LDS (fused eval_poly: one set, chunk 0)
    uint4 vi[PT], vf[PT], vs[PR], vv[PR];
    uint32_t ri = 0;
    BasisStager<K, NT> bs;
    bool basis = false;

    __device__ __forceinline__ void load(const PassArgs &A, const Ctx &c, uint32_t chunk) {
#ifdef RS_PROBE_SKIP_STAGE  // tools/pass_probe.hip: time a pass without table staging
        return;
#endif
        basis = A.tab_basis != 0;
        if (basis) {
            bs.load(*this, A, c, chunk);
            return;
        }
        const uint32_t tid = threadIdx.x;
        const uint32_t dI = A.ifft_delta + chunk * A.ifft_delta_step, dF = A.fft_delta + chunk * A.fft_delta_step;
        if (tabI || tabF) {
#pragma unroll
            for (int k = 0; k < PT; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kTw) {
                    if (tabI) vi[k] = twiddle_piece<K>(A, c, dI, t);
                    if (tabF) vf[k] = twiddle_piece<K>(A, c, dF, t);
                }
            }
        }
        if (tabS || tabV) {
            uint32_t f[PR];
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kRw) f[k] = ri_lds ? ri_lds[t / 5] : A.rowinfo[c.grow(t / 5, K) + chunk * A.n];
            }
            if (tid < (1u << K) && !ri_lds) ri = A.rowinfo[c.grow(tid, K) + chunk * A.n];
            const uint4 *lut4 = reinterpret_cast<const uint4 *>(A.lut);
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kRw) {
                    const uint32_t piece = t % 5, lf = f[k] & 0xFFFFu;
                    if (tabS) vs[k] = lut4[lf * 5u + piece];
                    if (tabV) vv[k] = lut4[(65535u - lf) * 5u + piece];
                }
            }
        }
    }

    __device__ __forceinline__ void store() const {
#ifdef RS_PROBE_SKIP_STAGE
        return;
#endif
        if (basis) {
            bs.store(*this);
            return;
        }
        const uint32_t tid = threadIdx.x;
        if (tabI || tabF) {
#pragma unroll
            for (int k = 0; k < PT; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kTw) {
                    if (tabI) reinterpret_cast<uint4 *>(tabI)[t] = vi[k];
                    if (tabF) reinterpret_cast<uint4 *>(tabF)[t] = vf[k];
                }
            }
        }
        if (tabS || tabV) {
            if (tid < (1u << K) && !ri_lds) rinfo[tid] = ri;
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const uint32_t t = tid + uint32_t(k) * NT;
                if (t < kRw) {
                    if (tabS) reinterpret_cast<uint4 *>(tabS)[t] = vs[k];
                    if (tabV) reinterpret_cast<uint4 *>(tabV)[t] = vv[k];
                }
            }
        }
    }
};

// Only the IFFT (or only the FFT) tables of one chunk: the per-chunk
// re-staging of multi-chunk passes.
template <int K, int NT>
__device__ __forceinline__ void stage_twiddles(const PassArgs &A, const Ctx &c, uint32_t chunk, uint32_t *tabI,
                                               uint32_t *tabF) {
    Stager<K, NT> st;
    st.tabI = tabI;
    st.tabF = tabF;
    st.load(A, c, chunk);
    st.store();
}

// Bit b (< 256) of a 4-word block mask: uniform words, per-lane selects.
__device__ __forceinline__ bool blk_bit(const uint64_t (&m)[4], uint32_t b) {
    const uint64_t w = b < 128 ? (b < 64 ? m[0] : m[1]) : (b < 192 ? m[2] : m[3]);
    return (w >> (b & 63u)) & 1u;
}

// Load the lane's rows (phase PH) of `chunk`.  SCALE: rows erased in the
// decode's erasure vector load as zero (checked in global rowinfo, so the
// load need not wait for staging).
template <int K, int LR, int SPL, int PH, bool SCALE, bool EVAL = false>
__device__ __forceinline__ void load_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, uint32_t (&lo)[1 << LR],
                                          uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    if (A.work_in && !SCALE) {
        // work rows: the lane's rows are r0 + i * 2^(start(PH) + a), so their
        // addresses are one 64-bit multiply-add plus a uniform step each
        const uint32_t r0 = c.grow(P::template lrow<PH>(c.g, 0), K) + chunk * A.n;
        const uint8_t *p0 = A.work_in + uint64_t(r0) * A.work_stride + c.pk_off;
        const uint64_t step = A.work_stride << (P::start(PH) + c.a);
        const bool per_row = A.blk_masks && !A.blk_uniform;
        const bool zero_set = A.blk_masks && A.blk_uniform &&
                              blk_bit(A.zero_in, __builtin_amdgcn_readfirstlane(r0 >> A.blk_shift));
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            uint32_t l = 0, h = 0;
            const uint32_t r = r0 + (uint32_t(i) << (P::start(PH) + c.a));
            if (c.pk_ok && !zero_set && !(per_row && blk_bit(A.zero_in, r >> A.blk_shift))) {
                const uint8_t *p = p0 + step * uint64_t(i);
                l = ld32(p);
                h = ld32(p + 32);
            }
            lo[i] = l;
            hi[i] = h;
        });
        return;
    }
    if (!A.work_in && A.nsrc == 1 && !SCALE) {  // one source matrix: the same, plus its row range
        const RowMap &m = A.src[0];
        const uint32_t r0 = c.grow(P::template lrow<PH>(c.g, 0), K) + chunk * A.n;
        const uint32_t d = 1u << (P::start(PH) + c.a);
        const uint8_t *p0 = m.base + int64_t(int32_t(r0 - m.row_begin)) * int64_t(m.stride) + c.pk_off;
        const uint64_t step = m.stride << (P::start(PH) + c.a);
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const uint32_t r = r0 + d * uint32_t(i);
            uint32_t l = 0, h = 0;
            if (c.pk_ok && r >= m.row_begin && r < m.row_end) {
                const uint8_t *p = p0 + step * uint64_t(i);
                l = ld_word(p, c.io);
                h = ld_word(p + c.io.hi_delta, c.io);
            }
            lo[i] = l;
            hi[i] = h;
        });
        return;
    }
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t r = pin<P::kUniform>(c.grow(P::template lrow<PH>(c.g, i), K) + chunk * A.n);
        const uint8_t *p = nullptr;
        if (A.work_in) {
            p = A.work_in + uint64_t(r) * A.work_stride;
        } else {
            if (r >= A.src[0].row_begin && r < A.src[0].row_end)
                p = A.src[0].base + uint64_t(r - A.src[0].row_begin) * A.src[0].stride;
            if (A.nsrc > 1 && r >= A.src[1].row_begin && r < A.src[1].row_end)
                p = A.src[1].base + uint64_t(r - A.src[1].row_begin) * A.src[1].stride;
        }
        if constexpr (EVAL) {  // fused eval_poly: not received = bit clear in the inline bitmap
            if (!((A.ev_received[(r >> 5) & 1u] >> (r & 31u)) & 1u)) p = nullptr;
        } else if (SCALE && (A.rowinfo[r] & 0x10000u)) {
            p = nullptr;
        }
        uint32_t l = 0, h = 0;
        if (p && c.pk_ok) {
            if (A.work_in) {
                l = ld32(p + c.pk_off);
                h = ld32(p + c.pk_off + 32);
            } else {
                l = ld_word(p + c.pk_off, c.io);
                h = ld_word(p + c.pk_off + c.io.hi_delta, c.io);
            }
        }
        lo[i] = l;
        hi[i] = h;
    });
}

template <int K, int LR, int SPL, int PH>
__device__ __forceinline__ void scale_rows(const Ctx &c, const uint32_t *tabS, uint32_t (&lo)[1 << LR],
                                           uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    uint32_t dep = 0;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        uint32_t off = P::template lrow<PH>(c.g, i) * 20u;
        if constexpr (P::kSerial) {
            if constexpr (P::kUniform) asm volatile("" : "+s"(off), "+v"(lo[i]), "+v"(hi[i]) : "v"(dep));
            else asm volatile("" : "+v"(off), "+v"(lo[i]), "+v"(hi[i]) : "v"(dep));
        }
        gf_mul4(lo[i], hi[i], tabS + off);
        dep = lo[i];
    });
}

template <int K, int LR, int SPL, int PH, bool REVEAL>
__device__ __forceinline__ void store_rows(const PassArgs &A, const Ctx &c, uint32_t chunk, const uint32_t *tabV,
                                           const uint32_t *rinfo, uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    if (A.work_out) {  // work rows: addresses as in load_rows
        const uint32_t r0 = c.grow(P::template lrow<PH>(c.g, 0), K) + chunk * A.n;
        uint8_t *p0 = A.work_out + uint64_t(r0) * A.work_stride + c.pk_off;
        const uint64_t step = A.work_stride << (P::start(PH) + c.a);
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const uint32_t r = r0 + (uint32_t(i) << (P::start(PH) + c.a));
            if (c.pk_ok && !(A.blk_masks && !A.blk_uniform && !blk_bit(A.keep_out, r >> A.blk_shift))) {
                uint8_t *p = p0 + step * uint64_t(i);
                st32(p, lo[i]);
                st32(p + 32, hi[i]);
            }
        });
        return;
    }
    if (!REVEAL) {  // destination matrix rows in [row_begin, row_end)
        const RowMap &m = A.dst;
        const uint32_t r0 = c.grow(P::template lrow<PH>(c.g, 0), K) + chunk * A.n;
        const uint32_t d = 1u << (P::start(PH) + c.a);
        uint8_t *p0 = const_cast<uint8_t *>(m.base) + int64_t(int32_t(r0 - m.row_begin)) * int64_t(m.stride) + c.pk_off;
        const uint64_t step = m.stride << (P::start(PH) + c.a);
        static_for<0, P::R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const uint32_t r = r0 + d * uint32_t(i);
            if (c.pk_ok && r >= m.row_begin && r < m.row_end) {
                uint8_t *p = p0 + step * uint64_t(i);
                st_word(p, lo[i], c.io);
                st_word(p + c.io.hi_delta, hi[i], c.io);
            }
        });
        return;
    }
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<PH>(c.g, i);
        const uint32_t r = pin<P::kUniform>(c.grow(j, K) + chunk * A.n);
        uint8_t *p = nullptr;
        uint32_t l = lo[i], h = hi[i];
        if (A.work_out) {
            p = A.work_out + uint64_t(r) * A.work_stride;
        } else if (r >= A.dst.row_begin && r < A.dst.row_end) {
            p = const_cast<uint8_t *>(A.dst.base) + uint64_t(r - A.dst.row_begin) * A.dst.stride;
            if constexpr (REVEAL) {
                if (rinfo[j] & 0x10000u) gf_mul4(l, h, tabV + j * 20u);
                else p = nullptr;
            }
        }
        if (p && c.pk_ok) {
            if (A.work_out) {
                st32(p + c.pk_off, l);
                st32(p + c.pk_off + 32, h);
            } else {
                st_word(p + c.pk_off, l, c.io);
                st_word(p + c.pk_off + c.io.hi_delta, h, c.io);
            }
        }
    });
}

// Block pruning of the decode's fused top pass (PassArgs::bfly_prune): local
// rows are blocks, zin / need the masks of zero-input / needed blocks.  The
// butterfly group of local row j at layer B covers the 2^(B+1) rows that share
// j's bits above B; an IFFT group is skipped when all of them are zero, an FFT
// group when none of them is needed (K <= 6: the masks are 64-bit).
struct Prune {
    uint64_t zin = 0, need = ~0ull;
};
template <bool IFFT, int B>
__device__ __forceinline__ bool group_live(const Prune &pr, uint32_t j) {
    constexpr uint64_t blk = B + 1 >= 6 ? ~0ull : (1ull << (1u << (B + 1))) - 1ull;
    const uint32_t base = j & ~((2u << B) - 1u);
    return IFFT ? ((pr.zin >> base) & blk) != blk : ((pr.need >> base) & blk) != 0;
}

// One butterfly layer on local bit B (global bit a + B), rows in phase PH.
template <int K, int LR, int SPL, int PH, int B, bool IFFT, bool PRUNE = false>
__device__ __forceinline__ void layer(const Ctx &c, const uint32_t *tab, uint32_t (&lo)[1 << LR],
                                      uint32_t (&hi)[1 << LR], const Prune &pr = Prune{}) {
    using P = Pass<K, LR, SPL>;
    constexpr int RB = B - P::start(PH);  // register bit
    static_assert(RB >= 0 && RB < LR, "bit not resident in this phase");
    static_assert(!PRUNE || (K <= 6 && P::kUniform), "block pruning: wave-uniform row groups, 64-bit masks");
    // Butterfly groups held by the lane: register index bits above RB.  One
    // 20-word table per group, read from LDS once for its 2^RB butterflies.
    uint32_t dep = 0;
    static_for<0, (P::R >> (RB + 1))>([&](auto gc) {
        constexpr int i0 = decltype(gc)::value << (RB + 1);
        if constexpr (PRUNE)
            if (!group_live<IFFT, B>(pr, P::template lrow<PH>(c.g, i0))) return;  // (uniform)
        uint32_t off = tw_slot<K>(B, P::template lrow<PH>(c.g, i0)) * 20u;
        if constexpr (P::kSerial) {  // one table in flight
            if constexpr (P::kUniform) asm volatile("" : "+s"(off) : "v"(dep));
            else asm volatile("" : "+v"(off) : "v"(dep));
        }
        const uint4 *t4 = reinterpret_cast<const uint4 *>(tab + off);
        uint32_t t[20];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint4 v = t4[q];
            t[4 * q] = v.x, t[4 * q + 1] = v.y, t[4 * q + 2] = v.z, t[4 * q + 3] = v.w;
        }
        static_for<0, (1 << RB)>([&](auto lc) {
            constexpr int i = i0 | decltype(lc)::value;
            constexpr int i2 = i | (1 << RB);
            if constexpr (P::kSerial) asm volatile("" : "+v"(lo[i]), "+v"(hi[i]), "+v"(lo[i2]), "+v"(hi[i2]) : "v"(dep));
            if constexpr (IFFT) ifft_bfly(lo[i], hi[i], lo[i2], hi[i2], t);
            else fft_bfly(lo[i], hi[i], lo[i2], hi[i2], t);
            dep = lo[i];
        });
    });
}

// A layer whose twiddle is zero (the top layer of a transform at skew offset 0,
// kZeroI / kZeroF; rs_mono.hip run_seq zero_top): both butterflies reduce to b ^= a.
template <int K, int LR, int SPL, int PH, int B>
__device__ __forceinline__ void xor_layer(uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    constexpr int RB = B - P::start(PH);
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (!((i >> RB) & 1)) {
            lo[i | (1 << RB)] ^= lo[i];
            hi[i | (1 << RB)] ^= hi[i];
        }
    });
}

// 2x2 transpose between lane rows 16 (LANE_BIT 4) or 32 (LANE_BIT 5) apart:
// the lane with lane bit clear keeps a and takes its partner's a as b, the
// partner keeps b and takes the a-lane's b as a (v_permlane{16,32}_swap).
template <int LANE_BIT>
__device__ __forceinline__ void lane_transpose(uint32_t &a, uint32_t &b) {
    if constexpr (LANE_BIT == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    } else {
        static_assert(LANE_BIT == 5, "in-wave row-group bits are lane bits 4 and 5");
        const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    }
}

// Move the rows from phase FROM to phase TO: through LDS (both planes at
// once), or -- 2 rows per lane, adjacent phases whose differing row-group bit
// lies inside the wave -- by a cross-lane transpose without LDS or barrier.
template <int K, int LR, int SPL, int FROM, int TO>
__device__ __forceinline__ void exchange(const Ctx &c, uint32_t *plane, uint32_t (&lo)[1 << LR],
                                         uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    constexpr uint32_t kPlane = uint32_t(P::SP) << K;
    if constexpr (FROM == TO) return;
    if constexpr (LR == 1 && (TO == FROM + 1 || FROM == TO + 1)) {
        // phases p and p+1 hold register bit p resp. p+1; the rows of lanes whose
        // row groups differ only in group bit p (row bit p+1 / p) are transposed
        constexpr int p = FROM < TO ? FROM : TO;
        if constexpr (SPL + p == 4 || SPL + p == 5) {
            lane_transpose<SPL + p>(lo[0], lo[1]);
            lane_transpose<SPL + p>(hi[0], hi[1]);
            return;
        }
    }
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t x = P::template lrow<FROM>(c.g, i) * P::SP + c.p;
        plane[x] = lo[i];
        plane[kPlane + x] = hi[i];
    });
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t x = P::template lrow<TO>(c.g, i) * P::SP + c.p;
        lo[i] = plane[x];
        hi[i] = plane[kPlane + x];
    });
}

// Formal derivative restricted to the set's local bits:
//   x[q] <- (mode 2 ? x[q] : 0) ^ XOR_{b < K, q_b = 0} x[q | 2^b]
template <int K, int LR, int SPL, int PH>
__device__ __forceinline__ void formal_derivative(const Ctx &c, uint32_t mode, uint32_t *plane,
                                                  uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    constexpr uint32_t kPlane = uint32_t(P::SP) << K;
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t x = P::template lrow<PH>(c.g, i) * P::SP + c.p;
        plane[x] = lo[i];
        plane[kPlane + x] = hi[i];
    });
    __syncthreads();
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t j = P::template lrow<PH>(c.g, i);
        uint32_t al = mode == 2 ? lo[i] : 0u, ah = mode == 2 ? hi[i] : 0u;
#pragma unroll
        for (int b = 0; b < K; ++b)
            if (!(j & (1u << b))) {
                const uint32_t x = (j | (1u << b)) * P::SP + c.p;
                al ^= plane[x];
                ah ^= plane[kPlane + x];
            }
        lo[i] = al;
        hi[i] = ah;
    });
}

template <int K, int LR, int SPL, int PH>
__device__ __forceinline__ void load_xor_rows(const PassArgs &A, const Ctx &c, uint32_t (&lo)[1 << LR],
                                              uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    static_for<0, P::R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t r = pin<P::kUniform>(c.grow(P::template lrow<PH>(c.g, i), K));
        const uint8_t *p = A.xor_in + uint64_t(r) * A.work_stride;
        uint32_t l = 0, h = 0;
        if (c.pk_ok) {
            l = ld32(p + c.pk_off);
            h = ld32(p + c.pk_off + 32);
        }
        lo[i] = l;
        hi[i] = h;
    });
}

// Twiddle tables of one layer held in registers: one 20-word table per
// butterfly group of the lane (at most R/2 groups, when the layer's bit is
// the lowest register bit).
template <int LR>
struct LayerTabs {
    uint32_t w[(1 << LR) / 2][20];
};

template <int K, int LR, int SPL, int PH, int B>
__device__ __forceinline__ void read_tables(const Ctx &c, const uint32_t *tab, LayerTabs<LR> &T) {
    using P = Pass<K, LR, SPL>;
    constexpr int RB = B - P::start(PH);
    static_for<0, (P::R >> (RB + 1))>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        const uint32_t off = tw_slot<K>(B, P::template lrow<PH>(c.g, g << (RB + 1))) * 20u;
        const uint4 *t4 = reinterpret_cast<const uint4 *>(tab + off);
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint4 v = t4[q];
            T.w[g][4 * q] = v.x, T.w[g][4 * q + 1] = v.y, T.w[g][4 * q + 2] = v.z, T.w[g][4 * q + 3] = v.w;
        }
    });
}

template <int K, int LR, int SPL, int PH, int B, bool IFFT>
__device__ __forceinline__ void apply_layer(const LayerTabs<LR> &T, uint32_t (&lo)[1 << LR],
                                            uint32_t (&hi)[1 << LR]) {
    using P = Pass<K, LR, SPL>;
    constexpr int RB = B - P::start(PH);
    static_for<0, (P::R >> (RB + 1))>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        static_for<0, (1 << RB)>([&](auto lc) {
            constexpr int i = (g << (RB + 1)) | decltype(lc)::value;
            constexpr int i2 = i | (1 << RB);
            if constexpr (IFFT) ifft_bfly(lo[i], hi[i], lo[i2], hi[i2], T.w[g]);
            else fft_bfly(lo[i], hi[i], lo[i2], hi[i2], T.w[g]);
        });
    });
}

// IFFT: bits ascending, starting in phase 0, ending in phase NPH-1.
// FFT: bits descending, starting in phase NPH-1, ending in phase 0.
// Narrow shapes (<= 4 rows per lane) read layer n+1's tables into registers
// while layer n runs, so the LDS latency hides behind the butterflies and
// the phase exchanges; wide shapes read one table at a time (registers).
// ZT: layer K-1 has a zero twiddle (kZeroI / kZeroF): no table, no multiply.
// PRUNE: block pruning of the decode's fused top pass (Prune, serial wide shapes).
template <int K, int LR, int SPL, bool IFFT, bool ZT = false, bool PRUNE = false>
__device__ __forceinline__ void transform(const Ctx &c, uint32_t *plane, const uint32_t *tab,
                                          uint32_t (&lo)[1 << LR], uint32_t (&hi)[1 << LR],
                                          const Prune &pr = Prune{}) {
    using P = Pass<K, LR, SPL>;
#ifdef RS_PROBE_SKIP_XFORM  // tools/pass_probe.hip: time a pass without its layers
    return;
#endif
    if constexpr (P::kSerial || K == 0) {
        static_for<0, K>([&](auto bc) {
            constexpr int n = decltype(bc)::value;
            constexpr int b = IFFT ? n : K - 1 - n;
            constexpr int prev = IFFT ? b - 1 : b + 1;
            constexpr int ph = P::phase_of(b);
            if constexpr (n > 0 && P::phase_of(prev) != ph)
                exchange<K, LR, SPL, P::phase_of(prev), ph>(c, plane, lo, hi);
            if constexpr (ZT && b == K - 1) xor_layer<K, LR, SPL, ph, b>(lo, hi);
            else layer<K, LR, SPL, ph, b, IFFT, PRUNE>(c, tab, lo, hi, pr);
        });
    } else {
        LayerTabs<LR> T[2];
        constexpr int b0 = IFFT ? 0 : K - 1;
        if constexpr (!(ZT && b0 == K - 1)) read_tables<K, LR, SPL, P::phase_of(b0), b0>(c, tab, T[0]);
        static_for<0, K>([&](auto bc) {
            constexpr int n = decltype(bc)::value;
            constexpr int b = IFFT ? n : K - 1 - n;
            constexpr int prev = IFFT ? b - 1 : b + 1;
            constexpr int next = IFFT ? b + 1 : b - 1;
            constexpr int ph = P::phase_of(b);
            if constexpr (n + 1 < K && !(ZT && next == K - 1))
                read_tables<K, LR, SPL, P::phase_of(next), next>(c, tab, T[(n + 1) & 1]);
            if constexpr (n > 0 && P::phase_of(prev) != ph)
                exchange<K, LR, SPL, P::phase_of(prev), ph>(c, plane, lo, hi);
            if constexpr (ZT && b == K - 1) xor_layer<K, LR, SPL, ph, b>(lo, hi);
            else apply_layer<K, LR, SPL, ph, b, IFFT>(T[n & 1], lo, hi);
        });
    }
}

template <int K, int LR, int SPL>
__device__ __forceinline__ Ctx make_ctx(const PassArgs &A, uint32_t bx) {
    using P = Pass<K, LR, SPL>;
    Ctx c;
    c.p = threadIdx.x & (P::SP - 1);
    c.g = threadIdx.x >> SPL;
    if constexpr (P::kUniform) c.g = __builtin_amdgcn_readfirstlane(c.g);
    const uint32_t slice = bx % A.slices;
    const uint32_t set = A.set_base + bx / A.slices;
    c.a = A.a;
    c.s_lo = set & ((1u << A.a) - 1u);
    c.s_hi = set >> A.a;
    const uint32_t pk = slice * P::SP + c.p;
    c.pk_ok = pk < A.packs;
    c.io = pack_io(A.fmt, pk);
    c.pk_off = c.io.lo;  // = (pk >> 3) * 64 + (pk & 7) * 4 for every pack
    return c;
}

// eval_poly of a single-pass decode (2^K <= 64 work rows, PassArgs::fused_eval)
// in wave 0, as k_eval_poly (rs_eval.hip; reference src/engine/utils.rs:20-31):
// erasure vector -> Walsh-Hadamard -> x lw_fold -> Walsh-Hadamard, all mod
// 65535, the butterfly partners across lanes (DPP / permlane swaps); row info
// into LDS.
template <int K>
__device__ __forceinline__ void pass_eval_poly(const PassArgs &A, uint32_t *rinfo, uint32_t lw) {
    static_assert((1 << K) <= int(kPassEvalRows), "one wave holds the points");
    const uint32_t i = threadIdx.x;
    if (i < 64) {
        constexpr uint32_t n = 1u << K;
        auto am = [](uint32_t a, uint32_t b) { const uint32_t s = a + b; return (s + (s >> 16)) & 0xFFFFu; };
        auto sm = [](uint32_t a, uint32_t b) { const uint32_t d = a - b; return (d + (d >> 16)) & 0xFFFFu; };
        const uint32_t e = i < n ? (A.ev_erased[i >> 5] >> (i & 31u)) & 1u : 0u;
        // high rate: v = e;  low rate: v = e - 1 on [0, end), 0 beyond  (mod 65535)
        uint32_t v = A.ev_low_rate ? (i < A.ev_end ? (e ? 0u : 65534u) : 0u) : e;
        auto walsh = [&]() {
            static_for<0, K>([&](auto hc) {
                constexpr int h = decltype(hc)::value;
                const uint32_t o = lane_xor<h>(v, i);
                v = (i >> h) & 1u ? sm(o, v) : am(v, o);
            });
        };
        walsh();
        const uint32_t p = v * lw;
        v = am(p & 0xFFFFu, p >> 16);
        if (A.ev_low_rate && i == 0) v = am(v, A.ev_lw0);
        walsh();
        const uint32_t rcv = i < n ? (A.ev_received[i >> 5] >> (i & 31u)) & 1u : 0u;
        if (i < n) rinfo[i] = v | (rcv ? 0u : 0x10000u);
    }
}

// The stager of the tables a pass block needs, targeting its LDS layout.
template <int K, int LR, int SPL, int FLAGS>
__device__ __forceinline__ Stager<K, Pass<K, LR, SPL>::kThreads> stager_for(uint32_t *lds) {
    using L = Lds<K, SPL, FLAGS>;
    constexpr bool DO_IFFT = FLAGS & kIfft, DO_FFT = FLAGS & kFft, MULTI_OUT = FLAGS & kMultiOut;
    constexpr bool SCALE = FLAGS & kScale, REVEAL = FLAGS & kReveal;
    Stager<K, Pass<K, LR, SPL>::kThreads> st;
    if constexpr (K > 0 && DO_IFFT) st.tabI = lds + L::oI;
    if constexpr (K > 0 && DO_FFT && !MULTI_OUT) st.tabF = lds + L::oF;
    if constexpr (SCALE) st.tabS = lds + L::oS;
    if constexpr (REVEAL) st.tabV = lds + L::oV;
    if constexpr (SCALE || REVEAL) st.rinfo = lds + L::oR;
    return st;
}

// One pass over workgroup-block (bx = set * slices + slice, by = chunk).
template <int K, int LR, int SPL, int FLAGS>
__device__ __forceinline__ void pass_body(const PassArgs &A, uint32_t bx, uint32_t by, uint32_t *lds) {
    using P = Pass<K, LR, SPL>;
    using L = Lds<K, SPL, FLAGS>;
    constexpr bool DO_IFFT = FLAGS & kIfft;
    constexpr bool DO_FFT = FLAGS & kFft;
    constexpr bool MULTI_IN = FLAGS & kMultiIn;    // XOR-fold IFFTs of A.in_chunks chunks
    constexpr bool MULTI_OUT = FLAGS & kMultiOut;  // FFT the same rows for A.out_chunks chunks
    constexpr bool SCALE = FLAGS & kScale;         // decode: scale received rows, zero erased ones
    constexpr bool FD = FLAGS & kFd;               // decode: formal derivative over local bits
    constexpr bool XOR_IN = FLAGS & kXorIn;        // decode: x ^= rows of A.xor_in
    constexpr bool REVEAL = FLAGS & kReveal;       // decode: store erased originals, unscaled
    constexpr bool EVAL = FLAGS & kEval;           // decode: eval_poly in the workgroup (one set, one chunk)
    constexpr bool ZI = FLAGS & kZeroI, ZF = FLAGS & kZeroF;  // zero-twiddle top layers
    static_assert(!(SCALE && MULTI_IN) && !(REVEAL && MULTI_OUT), "unsupported combination");
    static_assert(!(ZI && MULTI_IN) && !(ZF && MULTI_OUT), "zero-twiddle layers: one chunk per transform");
    static_assert(!EVAL || (SCALE && K <= 6), "fused eval_poly: single-pass decodes of <= 64 rows");
    constexpr int PL = P::NPH - 1;  // phase after an IFFT / before an FFT
    uint32_t *plane = lds;
    uint32_t *tabI = lds + L::oI, *tabF = lds + L::oF, *tabS = lds + L::oS, *tabV = lds + L::oV;
    uint32_t *rinfo = lds + L::oR;

    const Ctx c = make_ctx<K, LR, SPL>(A, bx);
    const uint32_t gchunk = by;
    // the decode's fused top pass: block pruning of its butterflies (PassArgs::bfly_prune)
    constexpr bool PRUNE = RS_PASS_BFLY_PRUNE && FD && DO_IFFT && DO_FFT && !REVEAL && !MULTI_IN && !MULTI_OUT &&
                           K <= 6 && P::kSerial && P::kUniform;
    Prune pr;
    if constexpr (PRUNE)
        if (A.bfly_prune) pr = Prune{A.zin_local, A.need_local};

    uint32_t lo[P::R], hi[P::R];
    uint32_t xl[XOR_IN ? P::R : 1], xh[XOR_IN ? P::R : 1];
    // loads first, then table staging: one barrier covers both latencies
    // fused eval_poly: its lw_fold values are the first load
    const uint32_t lwv = EVAL && threadIdx.x < (1u << K) ? uint32_t(A.ev_lw_fold[threadIdx.x]) : 0u;
    load_rows<K, LR, SPL, DO_IFFT ? 0 : PL, SCALE, EVAL>(A, c, A.in_chunk0 ? 0u : gchunk, lo, hi);
    if constexpr (XOR_IN) load_xor_rows<K, LR, SPL, PL>(A, c, xl, xh);
    {
        auto st = stager_for<K, LR, SPL, FLAGS>(lds);
        if constexpr (EVAL) {
            // twiddles in flight while eval_poly runs; then the row tables it indexes
            auto tw = st;
            tw.tabS = tw.tabV = nullptr;
            tw.load(A, c, gchunk);
            pass_eval_poly<K>(A, rinfo, lwv);
            tw.store();
            __syncthreads();
            st.tabI = st.tabF = nullptr;
            st.ri_lds = rinfo;
        }
        st.load(A, c, gchunk);
        st.store();
    }
    __syncthreads();
    if constexpr (SCALE) scale_rows<K, LR, SPL, 0>(c, tabS, lo, hi);

    if constexpr (DO_IFFT) {
        transform<K, LR, SPL, true, ZI, PRUNE>(c, plane, tabI, lo, hi, pr);
        if constexpr (MULTI_IN) {
            for (uint32_t ci = 1; ci < A.in_chunks; ++ci) {
                const uint32_t chunk = gchunk + ci;
                uint32_t tl[P::R], th[P::R];
                load_rows<K, LR, SPL, 0, false>(A, c, chunk, tl, th);
                __syncthreads();
                if constexpr (K > 0) stage_twiddles<K, P::kThreads>(A, c, chunk, tabI, nullptr);
                __syncthreads();
                transform<K, LR, SPL, true>(c, plane, tabI, tl, th);
                static_for<0, P::R>([&](auto ic) { lo[ic] ^= tl[ic]; hi[ic] ^= th[ic]; });
            }
        }
    }
    if constexpr (!DO_IFFT && MULTI_IN) {
        // rows already transformed per chunk (work_in, one chunk after another): XOR-fold
        for (uint32_t ci = 1; ci < A.in_chunks; ++ci) {
            uint32_t tl[P::R], th[P::R];
            load_rows<K, LR, SPL, PL, false>(A, c, gchunk + ci, tl, th);
            static_for<0, P::R>([&](auto ic) { lo[ic] ^= tl[ic]; hi[ic] ^= th[ic]; });
        }
    }
    // rows are now in phase PL

    if constexpr (FD) formal_derivative<K, LR, SPL, PL>(c, A.fd_mode, plane, lo, hi);
    if constexpr (XOR_IN) static_for<0, P::R>([&](auto ic) { lo[ic] ^= xl[ic]; hi[ic] ^= xh[ic]; });

    if constexpr (DO_FFT && !MULTI_OUT) {
        transform<K, LR, SPL, false, ZF, PRUNE>(c, plane, tabF, lo, hi, pr);
        store_rows<K, LR, SPL, 0, REVEAL>(A, c, gchunk, tabV, rinfo, lo, hi);
    } else if constexpr (DO_FFT) {
        for (uint32_t co = 0; co < A.out_chunks; ++co) {
            const uint32_t chunk = gchunk + co;
            uint32_t yl[P::R], yh[P::R];
            static_for<0, P::R>([&](auto ic) { yl[ic] = lo[ic]; yh[ic] = hi[ic]; });
            __syncthreads();
            if constexpr (K > 0) stage_twiddles<K, P::kThreads>(A, c, chunk, nullptr, tabF);
            __syncthreads();
            transform<K, LR, SPL, false>(c, plane, tabF, yl, yh);
            store_rows<K, LR, SPL, 0, false>(A, c, chunk, tabV, rinfo, yl, yh);
        }
    } else {
        store_rows<K, LR, SPL, PL, REVEAL>(A, c, gchunk, tabV, rinfo, lo, hi);
    }
}

// Occupancy: two 512-thread workgroups per CU at least; the encode's fused
// IFFT + FFT pass (the most butterflies per loaded row) is held to 6 waves per
// SIMD (<= 80 VGPRs) so that three of its workgroups share a CU: one's row
// loads and stores overlap the others' layers.
template <int LR, int FLAGS>
constexpr int pass_waves_per_eu() {
    return (FLAGS & ~(kZeroI | kZeroF)) == (kIfft | kFft) && LR == 3 ? 6 : 2;
}

template <int K, int LR, int SPL, int FLAGS>
__global__ void __launch_bounds__(1 << (K - LR + SPL), (pass_waves_per_eu<LR, FLAGS>())) k_pass(const PassArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    pass_body<K, LR, SPL, FLAGS>(A, blockIdx.x, blockIdx.y, lds);
}

template <int K, int LR, int SPL, int F>
hipError_t launch_f(const PassArgs &A, hipStream_t s) {
    using P = Pass<K, LR, SPL>;
    const size_t lds = Lds<K, SPL, F>::bytes();
    static std::atomic<uint64_t> attr_devs{0};  // devices whose attribute is set
    if (lds > 65536) {
        hipError_t e = lds_attr_once(attr_devs, reinterpret_cast<const void *>(&k_pass<K, LR, SPL, F>), int(lds));
        if (e != hipSuccess) return e;
    }
    PassArgs B = A;
    B.slices = (A.packs + P::SP - 1) / P::SP;
    const uint32_t total = B.slices * B.nsets;
    dim3 grid(total, B.grid_chunks);
    k_pass<K, LR, SPL, F><<<grid, P::kThreads, lds, s>>>(B);
    snprintf(launch_name_buf(), kLaunchNameBytes, "k_pass<%d, %d, %d, %d>", K, LR, SPL, F);
    return hipGetLastError();
}

template <int K, int LR, int SPL>
hipError_t launch_k(int flags, const PassArgs &A, hipStream_t s) {
    if (A.in_chunks > 1) flags |= kMultiIn;
    if (A.out_chunks > 1) flags |= kMultiOut;
    if (A.load_scale) flags |= kScale;
    if (A.fd_mode) flags |= kFd;
    if (A.xor_in) flags |= kXorIn;
    if (A.reveal) flags |= kReveal;
    if (A.fused_eval) {
        if (A.nsets != 1 || A.set_base || A.a || A.grid_chunks != 1 || (1u << K) > kPassEvalRows)
            return hipErrorInvalidValue;
        flags |= kEval;
    }
    constexpr int I = kIfft, F = kFft;
    // zero-twiddle top layers (RS_MONO_ZERO_TOP): the pass holds the transform's top
    // bit (a + K = log2 n) and every chunk of the launch has skew offset 0; the
    // fused top passes of encodes (HighRate: FFT; LowRate: IFFT) and decodes (both)
    // have variants for it
    if (RS_MONO_ZERO_TOP && K > 0 && A.n > 1 && A.a + uint32_t(K) == uint32_t(__builtin_ctz(A.n))) {
        const bool one = A.grid_chunks == 1;
        const bool zi = (flags & I) && A.ifft_delta == 0 && A.in_chunks == 1 && (one || A.ifft_delta_step == 0);
        const bool zf = (flags & F) && A.fft_delta == 0 && A.out_chunks == 1 && (one || A.fft_delta_step == 0);
        if (flags == (I | F) && zf && !zi) return launch_f<K, LR, SPL, I | F | kZeroF>(A, s);
        // LowRate: the IFFT of the originals at skew offset 0, FFTs at c n + n
        if (flags == (I | F) && zi && !zf) return launch_f<K, LR, SPL, I | F | kZeroI>(A, s);
        if (flags == (I | F | kMultiOut) && zi) return launch_f<K, LR, SPL, I | F | kMultiOut | kZeroI>(A, s);
        if (flags == (I | F | kFd) && zi && zf) return launch_f<K, LR, SPL, I | F | kFd | kZeroI | kZeroF>(A, s);
    }
    switch (flags) {
        // encode / engine
        case I: return launch_f<K, LR, SPL, I>(A, s);
        case F: return launch_f<K, LR, SPL, F>(A, s);
        case I | F: return launch_f<K, LR, SPL, I | F>(A, s);
        case I | kMultiIn: return launch_f<K, LR, SPL, I | kMultiIn>(A, s);
        case I | F | kMultiIn: return launch_f<K, LR, SPL, I | F | kMultiIn>(A, s);
        case I | F | kMultiOut: return launch_f<K, LR, SPL, I | F | kMultiOut>(A, s);
        case F | kMultiOut: return launch_f<K, LR, SPL, F | kMultiOut>(A, s);
        case F | kMultiIn: return launch_f<K, LR, SPL, F | kMultiIn>(A, s);
        // decode: single pass, IFFT passes, fused top, FFT passes (middle / last)
        case I | F | kScale | kFd | kReveal: return launch_f<K, LR, SPL, I | F | kScale | kFd | kReveal>(A, s);
        case I | F | kScale | kFd | kReveal | kEval:
            if constexpr (K <= 6) return launch_f<K, LR, SPL, I | F | kScale | kFd | kReveal | kEval>(A, s);
            return hipErrorInvalidValue;
        case I | kScale: return launch_f<K, LR, SPL, I | kScale>(A, s);
        case I | F | kFd: return launch_f<K, LR, SPL, I | F | kFd>(A, s);
        case F | kFd | kXorIn: return launch_f<K, LR, SPL, F | kFd | kXorIn>(A, s);
        case F | kFd | kXorIn | kReveal: return launch_f<K, LR, SPL, F | kFd | kXorIn | kReveal>(A, s);
        default: return hipErrorInvalidValue;
    }
}

// Two shapes per K: "wide" (8 rows per lane; 64-pack slices up to K = 6, 32
// at K = 7 and 16 at K = 8, so that a workgroup stays at 512 threads and at
// most 80 KiB of LDS and two of them share a CU: one's loads and stores
// overlap the other's butterflies -- measured in profiles/r01k) for matrices
// that fill the chip, "narrow" (16..32-pack slices, 2 rows per lane -- 4 at
// K = 8 -- in-wave phase changes by lane transposes) to spread small matrices
// over more workgroups and waves.
template <int K>
hipError_t launch_shape(bool narrow, int flags, const PassArgs &A, hipStream_t s) {
    // (16 rows per lane at K = 7, 8 -- two phases, one exchange -- measured slower at
    // configs 3 and 5: 1 workgroup per CU; tools/ab_variant.sh)
    constexpr int LRW = K < 3 ? K : 3;
    constexpr int SPLW = K >= 8 ? 4 : K == 7 ? 5 : 6;
    if constexpr (K >= 2) {
        constexpr int LRN = K >= 8 ? 2 : 1;
        constexpr int SPLN = 6 - (K - LRN) > 4 ? 6 - (K - LRN) : 4;
        if (narrow) return launch_k<K, LRN, SPLN>(flags, A, s);
    }
    return launch_k<K, LRW, SPLW>(flags, A, s);
}


__global__ void k_mul(uint8_t *rows, uint64_t packs, const uint32_t *t) {
    const uint64_t pk = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (pk >= packs) return;
    uint32_t *p = reinterpret_cast<uint32_t *>(rows + (pk >> 3) * 64 + (pk & 7) * 4);
    uint32_t l = p[0], h = p[8];
    gf_mul4(l, h, t);
    p[0] = l;
    p[8] = h;
}

__global__ void k_formal_derivative(const uint8_t *in, uint8_t *out, uint32_t rows, uint64_t words_per_row) {
    const uint64_t wi = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint32_t q = blockIdx.y;
    if (wi >= words_per_row) return;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(in);
    uint32_t acc = src[uint64_t(q) * words_per_row + wi];
    for (uint32_t b = 1; b < rows; b <<= 1)
        if (!(q & b) && (q | b) < rows) acc ^= src[uint64_t(q | b) * words_per_row + wi];
    reinterpret_cast<uint32_t *>(out)[uint64_t(q) * words_per_row + wi] = acc;
}

}  // namespace

hipError_t launch_pass(int K, int flags, const PassArgs &A, hipStream_t s) {
    // narrow slices when the wide shape's slices leave the chip under-filled
    const uint32_t wide_packs = K >= 8 ? 16 : K == 7 ? 32 : 64;
    const uint64_t wide_groups = uint64_t(A.nsets) * ((A.packs + wide_packs - 1) / wide_packs) * A.grid_chunks;
// the narrow shape where the wide one would leave the chip under-filled: below
// 1024 workgroups, 512 at K >= 7 (16384:16384 x 1 KiB encode 62.3 -> 53.2 us; the
// K <= 6 passes lost with 512, profiles/r04a/pass_narrow_threshold.txt)
#ifndef RS_PASS_NARROW_BELOW
#define RS_PASS_NARROW_BELOW (K >= 7 ? 512 : 1024)
#endif
    const bool narrow = wide_groups < uint64_t(RS_PASS_NARROW_BELOW);
    switch (K) {
        case 0: return launch_shape<0>(narrow, flags, A, s);
        case 1: return launch_shape<1>(narrow, flags, A, s);
        case 2: return launch_shape<2>(narrow, flags, A, s);
        case 3: return launch_shape<3>(narrow, flags, A, s);
        case 4: return launch_shape<4>(narrow, flags, A, s);
        case 5: return launch_shape<5>(narrow, flags, A, s);
        case 6: return launch_shape<6>(narrow, flags, A, s);
        case 7: return launch_shape<7>(narrow, flags, A, s);
        case 8: return launch_shape<8>(narrow, flags, A, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_mul(uint8_t *rows, uint64_t blocks, const uint32_t *t, hipStream_t s) {
    const uint64_t packs = blocks * 8;
    if (!packs) return hipSuccess;
    k_mul<<<dim3(uint32_t((packs + 255) / 256)), 256, 0, s>>>(rows, packs, t);
    return hipGetLastError();
}

hipError_t launch_formal_derivative(const uint8_t *in, uint8_t *out, uint32_t rows, uint64_t row_bytes, hipStream_t s) {
    const uint64_t words = row_bytes / 4;
    if (!rows || !words) return hipSuccess;
    k_formal_derivative<<<dim3(uint32_t((words + 255) / 256), rows), 256, 0, s>>>(in, out, rows, words);
    return hipGetLastError();
}

}  // namespace rs
