// Column kernel ("mono") of the MI355X Reed-Solomon engine.
//
// One workgroup owns every one of the n = 2^L transform rows of ONE pack (4
// GF(2^16) elements: 4 low bytes at block offset 4p, 4 high bytes at 32 + 4p,
// reference layout src/algorithm.md:18-31).  Every engine op is column-wise
// (src/engine/utils.rs:35-43, src/engine/engine_naive.rs:107-146), so the
// whole encode -- IFFT (engine_naive.rs:75-105), chunk XOR-fold / replicate
// (rate_high.rs:56-74, rate_low.rs:59-78), FFT (engine_naive.rs:43-73) -- or
// decode (rate_high.rs:172-254) runs inside one workgroup: there is no
// cross-workgroup hand-off, which is what bounds the multi-pass kernels at
// small shard matrices (DESIGN.md "Column kernel").
//
// Rows live in registers: a lane holds R = 2^LR rows; row-index bits are
// spread over register bits, the 6 lane bits and the wave bits.  A butterfly
// layer on row bit x needs x in a register bit; it gets there by a 2x2
// register/lane transpose (DPP or v_permlane{16,32}_swap -- no
// LDS traffic, no barrier) or, for wave bits, by one LDS remap of the whole
// column (twice per transform pair).  The plan (which bit sits where before
// every op) is computed at compile time.
//
// Twiddle tables are read straight from layer-ordered images (rs_device.hpp)
// into registers, one layer ahead of use, so table latency hides behind the
// butterflies of the current layer.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>

#include "rs_device.hpp"
#include "rs_gf.hpp"

namespace rs {
namespace {

#ifdef RS_MONO_STAMPS  // tools/mono_probe.hip: per-workgroup timestamps
__device__ uint64_t g_mono_stamps[4096][24];
#ifdef RS_MONO_STAMP_WAIT  // each stamp first waits for the wave's outstanding memory ops
#define RS_MSTAMP_WAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else  // the time the wave's instruction stream reaches the stamp
#define RS_MSTAMP_WAIT() asm volatile("" ::: "memory")
#endif
#define RS_MSTAMP(i)                                                                                 \
    do {                                                                                             \
        RS_MSTAMP_WAIT();                                                                            \
        if (threadIdx.x == blockDim.x - 64 && blockIdx.x + blockIdx.y * gridDim.x < 4096) g_mono_stamps[blockIdx.x + blockIdx.y * gridDim.x][i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define RS_MSTAMP(i)
#endif

// ---------------------------------------------------------------------------
// compile-time plan

struct Map {
    int reg[3];   // row bit held by register-index bit s
    int lane[6];  // row bit held by lane bit j
    int wave[4];  // row bit held by wave bit k
};
enum : int { kOpLayer = 1, kOpXpose = 2, kOpRemap = 3 };
struct Op {
    int kind, bit, rs, ls;  // layer on `bit` (register bit rs) / swap register bit rs with lane bit ls
};
constexpr int kMaxOps = 64;
struct Seq {
    int count = 0;
    Op ops[kMaxOps] = {};
    Map maps[kMaxOps + 1] = {};  // maps[i]: placement before op i; maps[count]: final
};

constexpr int find_reg(const Map &m, int LR, int x) {
    for (int s = 0; s < LR; ++s)
        if (m.reg[s] == x) return s;
    return -1;
}
constexpr int find_lane(const Map &m, int x) {
    for (int j = 0; j < 6; ++j)
        if (m.lane[j] == x) return j;
    return -1;
}
constexpr int next_use(const int *bits, int nb, int from, int x) {
    for (int t = from; t < nb; ++t)
        if (bits[t] == x) return t;
    return 1 << 20;
}
constexpr void push(Seq &s, Op op, const Map &after) {
    s.ops[s.count] = op;
    ++s.count;
    s.maps[s.count] = after;
}

// Butterfly layers on `bits` in order; a bit not in a register is swapped in
// from its lane bit, evicting the register bit used furthest in the future.
constexpr void layers(Seq &s, Map &m, int LR, const int *bits, int nb) {
    for (int t = 0; t < nb; ++t) {
        const int x = bits[t];
        int rs = find_reg(m, LR, x);
        if (rs < 0) {
            const int j = find_lane(m, x);
            int far = -1;
            for (int q = 0; q < LR; ++q) {
                const int u = next_use(bits, nb, t + 1, m.reg[q]);
                if (u > far) far = u, rs = q;
            }
            const int tmp = m.reg[rs];
            m.reg[rs] = m.lane[j];
            m.lane[j] = tmp;
            push(s, Op{kOpXpose, x, rs, j}, m);
        }
        push(s, Op{kOpLayer, x, rs, 0}, m);
    }
}

// Placement of a segment: in-wave bits [lo, lo + IW), wave bits the rest.
// Registers take the first bits of `order`; lane bits the next ones, cheapest
// transposes (permlane swaps: lane bits 5, 4; DPP: 0, 1, 3; two DPP moves: 2) first.
constexpr Map seg_map(int L, int LR, int lo, const int *order, int no) {
    const int IW = LR + 6;
    int pri[16] = {}, np = 0;
    for (int t = 0; t < no; ++t) {
        const int x = order[t];
        bool seen = x < lo || x >= lo + IW;
        for (int q = 0; q < np; ++q) seen = seen || pri[q] == x;
        if (!seen) pri[np++] = x;
    }
    for (int x = lo; x < lo + IW; ++x) {
        bool seen = false;
        for (int q = 0; q < np; ++q) seen = seen || pri[q] == x;
        if (!seen) pri[np++] = x;
    }
    const int pref[6] = {5, 4, 0, 1, 3, 2};
    Map m{};
    for (int s = 0; s < 3; ++s) m.reg[s] = s < LR ? pri[s] : -1;
    for (int j = 0; j < 6; ++j) m.lane[pref[j]] = pri[LR + j];
    int k = 0;
    for (int x = 0; x < L; ++x)
        if (x < lo || x >= lo + IW) m.wave[k++] = x;
    for (; k < 4; ++k) m.wave[k] = -1;
    return m;
}

// SPLIT (decodes whose restored rows lie in one half of the 2^L work rows):
// the top row bit L-1 stays a wave bit throughout, so each half is a 2^(L-1)
// row transform of its own waves; the IFFT stops below layer L-1, the top
// layers of both transforms and the formal derivative's cross-half term run
// in one exchange (split_top), and only the half holding restored rows runs
// the rest of the FFT.
// SP bit 1 (FLOW, decodes): the FFT leaves the top placement after layer IW
// instead of WB, so its layers IW-1..0 run with the low bits in-wave -- each
// wave then holds 2^IW consecutive rows, the waves without restored rows stop
// there, and those layers reuse the IFFT's phase-1 tables
template <int L, int LR, int SP = 0>
struct Plan {
    static constexpr bool SPLIT = (SP & 1) != 0, FLOW = (SP & 2) != 0;
    static constexpr int IW = LR + 6, WB = L - IW - (SPLIT ? 1 : 0), R = 1 << LR;
    static_assert(WB >= 0 && L - IW <= 4, "column kernel: 6 lane bits + LR register bits + up to 4 wave bits");
    static_assert(!SPLIT || WB >= 1, "split plan: at least one wave bit below the top bit");
    static constexpr int TOP = SPLIT ? L - 1 : L;  // layers [0, TOP) run in the sequences
    // lowest FFT layer of the top placement (the FFT's low segment: layers FLO-1..0)
    static constexpr int FLO = FLOW && WB > 0 ? IW : WB;

    static constexpr Seq make_ifft() {
        Seq s{};
        int bits[16] = {}, order[32] = {}, no = 0;
        if (WB == 0 && !SPLIT) {
            for (int x = 0; x < L; ++x) order[no++] = x;
            for (int x = L - 1; x >= 0; --x) order[no++] = x;
            Map m = seg_map(L, LR, 0, order, no);
            s.maps[0] = m;
            for (int x = 0; x < L; ++x) bits[x] = x;
            layers(s, m, LR, bits, L);
            return s;
        }
        // segment A: IFFT layers 0..IW-1 with the low bits in-wave
        for (int x = 0; x < IW; ++x) order[no++] = x, bits[x] = x;
        Map m = seg_map(L, LR, 0, order, no);
        s.maps[0] = m;
        layers(s, m, LR, bits, IW);
        // segment B: the top IW bits (below bit L-1 when SPLIT) in-wave: IFFT
        // layers IW..TOP-1 (then FFT TOP-1..WB)
        no = 0;
        for (int x = IW; x < TOP; ++x) order[no++] = x;
        for (int x = TOP - 1; x >= WB; --x) order[no++] = x;
        m = seg_map(L, LR, WB, order, no);
        push(s, Op{kOpRemap, -1, 0, 0}, m);
        for (int x = IW; x < TOP; ++x) bits[x - IW] = x;
        layers(s, m, LR, bits, TOP - IW);
        return s;
    }
    static constexpr Seq ifft = make_ifft();

    static constexpr Seq make_fft() {
        Seq s{};
        int bits[16] = {}, order[16] = {}, no = 0;
        Map m = ifft.maps[ifft.count];
        s.maps[0] = m;
        const int stop = FLO;  // FFT layers TOP-1..stop in the IFFT's final placement
        for (int x = TOP - 1; x >= stop; --x) bits[TOP - 1 - x] = x;
        layers(s, m, LR, bits, TOP - stop);
        if (WB == 0) return s;
        // segment C: the low IW bits in-wave again, FFT layers FLO-1..0
        for (int x = FLO - 1; x >= 0; --x) order[no++] = x;
        m = seg_map(L, LR, 0, order, no);
        push(s, Op{kOpRemap, -1, 0, 0}, m);
        for (int x = FLO - 1; x >= 0; --x) bits[FLO - 1 - x] = x;
        layers(s, m, LR, bits, FLO);
        return s;
    }
    static constexpr Seq fft = make_fft();
};

template <int L, int LR, bool FFT, int SPLIT = 0>
struct SeqOf {
    static constexpr const Seq &v = FFT ? Plan<L, LR, SPLIT>::fft : Plan<L, LR, SPLIT>::ifft;
};

constexpr int layer_ordinal(const Seq &s, int i) {
    int k = 0;
    for (int q = 0; q < i; ++q) k += s.ops[q].kind == kOpLayer;
    return k;
}

// ---------------------------------------------------------------------------
// device helpers

// Row index of register i under placement maps[I] of sequence S.
template <typename S, int I>
__device__ __forceinline__ uint32_t lane_rows(uint32_t lane, uint32_t wave) {
    constexpr Map m = S::v.maps[I];
    uint32_t r = 0;
    static_for<0, 6>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        r |= ((lane >> j) & 1u) << m.lane[j];
    });
    static_for<0, 4>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if constexpr (m.wave[k] >= 0) r |= ((wave >> k) & 1u) << m.wave[k];
    });
    return r;
}
template <typename S, int I, int LR>
__device__ __forceinline__ constexpr uint32_t reg_rows(int i) {
    constexpr Map m = S::v.maps[I];
    uint32_t r = 0;
    for (int s = 0; s < LR; ++s) r |= uint32_t((i >> s) & 1) << m.reg[s];
    return r;
}

// LDS column plane: low words at [0, n), high words at [n, 2n); the index is
// XOR-swizzled inside 32-word runs against strided lane access.
template <int L>
__device__ __forceinline__ uint32_t swz(uint32_t r) {
    return r ^ ((r >> 5) & 31u);
}

// 2x2 transpose of (register pair, lane bit J): the lane with bit J clear ends
// with (a, partner's a), its partner with (a-lane's b, b).
template <int J>
__device__ __forceinline__ void xpose(uint32_t &a, uint32_t &b, uint32_t lane) {
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

// Pack format: E = 4 elements per pack (a row is a low-byte word and a
// high-byte word, 20-word tables, rs_gf.hpp gf_muladd4) or E = 2 (a row is one
// word [lo0 lo1 hi0 hi1], 16-word tables, gf_muladd2): the 2-element form gives
// a shard matrix twice the workgroups (packs = shard_bytes / 4), for matrices
// whose 4-element packs leave CUs idle.
template <int E>
struct Fmt {
    static_assert(E == 4 || E == 2, "pack format");
    static constexpr int kTW = E == 4 ? 20 : 16;  // table words
    static constexpr uint32_t kPC = kTW / 4;      // 16-byte pieces per table
    static constexpr bool kHi = E == 4;           // rows have a separate high-byte word
};

template <int L, int LR, int E = 4>
struct Col {
    static constexpr int R = 1 << LR;
    static constexpr uint32_t n = 1u << L;
    uint32_t lo[R], hi[E == 4 ? R : 1];
};

// Index of register pair (i, i | 2^s) among the pairs of register bit s.
constexpr int pair_of(int i, int s) { return (i & ((1 << s) - 1)) | ((i >> (s + 1)) << s); }

// The perm table of the butterfly group of row `row` at layer x.
__device__ __forceinline__ void load_tab(const uint32_t *img, int L, int x, uint32_t row, uint32_t (&t)[20]) {
    const uint32_t n = 1u << L;
    const uint32_t slot = n - (n >> x) + (row >> (x + 1));
#ifdef RS_MONO_FAKE_TABS  // tools/mono_probe.hip: tables without memory traffic
    for (int q = 0; q < 20; ++q) t[q] = slot * 0x01010101u + q;
    return;
#endif
    const uint4 *p = reinterpret_cast<const uint4 *>(img) + slot * 5u;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const uint4 v = p[q];
        t[4 * q] = v.x, t[4 * q + 1] = v.y, t[4 * q + 2] = v.z, t[4 * q + 3] = v.w;
    }
}

// Table source: the layer-ordered image in global memory (through L1).
struct GlobalTabs {
    const uint32_t *img;
    template <int L, int LR, typename S, int I, int PH>
    __device__ __forceinline__ void get(int x, uint32_t row, uint32_t (&t)[20]) const {
        load_tab(img, L, x, row, t);
    }
};

// Basis images (2-element packs, RS_MONO_BASIS, default off): the staging loads a
// table's 16 basis products (8 words, rs_codec.cpp basis_images) instead of its 16
// words, and builds the table in LDS.  Multiplication by a constant is GF(2)-linear,
// so the four lookups of 2-bit field f are {0, a, b, a ^ b} with a, b its two basis
// products; basis word 2f = a | b << 16 of the low byte's field f (A_f), word 2f + 1
// the high byte's (C_f), so one 16-byte basis piece (A_f, C_f, A_f+1, C_f+1) makes
// table pieces f and f + 1 (gf_tables.cpp fill_perm2: direct words [0, a_lo, b_lo,
// (a^b)_lo] and [0, c_hi, d_hi, (c^d)_hi], cross words with the other bytes), two
// v_perm_b32 and an XOR per word pair.  Half the staging's L2 requests: k_chunks
// 1000:100 x 1 KiB 10.8 -> 5.9 us per launch (profiles/r05g/chunks_basis.txt), but
// k_mono unchanged or slower: headline encode 7.92 / 7.96 -> 7.94 / 7.94 us, decode
// 2^11 rows 1 % 13.47 / 13.42 -> 13.63 / 13.62 us (profiles/r05h/basis_ab.txt), so
// RS_MONO_BASIS (rs_device.hpp) is off: 1 builds k_mono with it (the host then
// hands it basis images, rs_codec.cpp mono_args).

template <int L, int LR, int SP = 0, int E = 4>
struct Stage {
    static constexpr bool SPLIT = Plan<L, LR, SP>::SPLIT;
    static constexpr int FLO = Plan<L, LR, SP>::FLO;
    static constexpr int TW = Fmt<E>::kTW;
    static constexpr uint32_t PC = Fmt<E>::kPC;
    static constexpr bool kBasis = E == 2 && RS_MONO_BASIS;
    static constexpr uint32_t LPC = kBasis ? 2 : PC;  // image pieces per table (basis images: 8 words)
    // write image piece q (of a region's image pieces) into the region's LDS slots
    template <typename AT>
    static __device__ __forceinline__ void put(uint32_t *region, uint32_t q, const uint4 &v, AT at) {
        if constexpr (kBasis) {
            const uint32_t p0 = (q >> 1) * PC + (q & 1u) * 2u;  // table piece of field 2 (q & 1)
            uint4 a, b;
            basis2_expand(v, a, b);
            reinterpret_cast<uint4 *>(region)[at(p0)] = a;
            reinterpret_cast<uint4 *>(region)[at(p0 + 1)] = b;
        } else {
            reinterpret_cast<uint4 *>(region)[at(q)] = v;
        }
    }
    // LDS slot of a table: 20 words in both formats.  A 2-element table is 16
    // words, and slots of 16 words (64 B, a quarter of the banks) would put lanes
    // that read tables t and t + 4 on the same banks; 20-word slots cycle through
    // all 16 four-bank groups (MI355X guide "LDS": ds_read_b128 lane groups)
    static constexpr int SW = 20;
    static constexpr uint32_t SPC = SW / 4;  // 16-byte pieces per slot
    // Within a layer, group g's table sits at slot sg(g) = g ^ ((g >> 1) & 15) of the
    // layer's range.  The plan puts row bits 3 and 4 (and, in the FFT's top phase,
    // similar pairs) on lane bits of one ds_read_b128 lane group, so layers 0 and 1
    // read groups 2 and 4 slots apart on the same banks; the Gray-code swizzle
    // spreads them (a model of every table read of the plans, tools/lds_bank_model.py,
    // gives conflict-free reads for L = 8..11).  Measured (profiles/r02h/ab_gray): the
    // 2-element decode's conflict cycles 708K -> 566K per launch and -0.2 us, but the
    // 4-element encode's 106K -> 204K (the permuted staging writes and the phase-3 XOR
    // pass conflict instead) and +0.2 us, so only the 2-element format uses it
    static constexpr bool kGray = E == 2;
    static __device__ __forceinline__ uint32_t sg(uint32_t g) { return kGray ? g ^ ((g >> 1) & 15u) : g; }
    // slot of table t of a region sequence of 2^k - 1 tables, layers largest first
    // (layer of size 2^m starts at 2^k - 2^(m+1), a multiple of 2^m)
    static __device__ __forceinline__ uint32_t sq(uint32_t t, uint32_t k) {
        if constexpr (!kGray) return t;
        const uint32_t y = (1u << k) - t;  // 2^m < y <= 2^(m+1)
        const uint32_t mask = y <= 1u ? 0u : (1u << (31 - __builtin_clz(y - 1u))) - 1u;
        return t ^ (((t & mask) >> 1) & 15u);
    }
    // LDS position (16-byte units) of piece q of table slot (q / PC) -> f(q / PC)
    template <typename F>
    static __device__ __forceinline__ uint32_t at(uint32_t q, F f) {
        const uint32_t t = q / PC;
        return f(t) * SPC + (q - t * PC);
    }
    // the phase-1 / -3 region (layers B0..IW-1), its layer-0 turn (B0), the shared region
    static __device__ __forceinline__ uint32_t at1(uint32_t q) {
        return at(q, [](uint32_t t) { return sq(t, uint32_t(IW - B0)); });
    }
    static __device__ __forceinline__ uint32_t at0(uint32_t q) { return at(q, [](uint32_t t) { return sg(t); }); }
    static __device__ __forceinline__ uint32_t atS(uint32_t q) {
        return at(q, [](uint32_t t) {
            if (t < kShI) return sq(t, uint32_t(L - IW));
            if (t < kShI + kShF) return kShI + sq(t - kShI, uint32_t(L - FLO));
            return t;  // D tables: one per layer
        });
    }
    static constexpr int IW = LR + 6, WB = L - IW - (SPLIT ? 1 : 0);
    static constexpr uint32_t n = 1u << L, W = 1u << IW;
    // layers of the last (FFT) in-wave phase
    static constexpr int NB3 = WB > 0 ? FLO : L;
    // B0 = 1: layer 0 of phases 1 and 3 (one table per butterfly) takes turns
    // with the other layers in the private regions, so they fit LDS at L = 11
#ifndef RS_MONO_B0_MIN_L
#define RS_MONO_B0_MIN_L 11
#endif
    static constexpr int B0 = L >= RS_MONO_B0_MIN_L ? 1 : 0;
    // tables per wave region; with B0 the region first holds layer 0's W/2
    // tables, then (written over them, see run_seq's hook) the layers above
    static constexpr uint32_t kPriv = B0 ? (W >> 1) : W - 1;
    static constexpr uint32_t kUp = (W >> B0) - 1;                   // tables of phase 1 (layer 0 apart)
    static constexpr uint32_t kP3 = (W >> B0) - (W >> NB3);          // tables of phase 3 (layer 0 apart)
    static constexpr uint32_t kL0 = W >> 1;                          // layer-0 tables of a wave region
    static constexpr uint32_t kShI = WB > 0 ? (n >> IW) - 1 : 0;     // shared: IFFT layers IW..L-1
    static constexpr uint32_t kShF = WB > 0 ? (n >> FLO) - 1 : 0;    // shared: FFT layers FLO..L-1
    static constexpr uint32_t kShared = kShI + kShF;
    static constexpr uint32_t kWaves = 1u << (L - LR - 6);
    static constexpr uint32_t plane_words = (E == 4 ? 2 : 1) * n;
    static constexpr uint32_t words = plane_words + (kShared + kWaves * kPriv) * SW;
    // encode (IFFT and FFT on different skew offsets t_i, t_f): phase 3's tables
    // are phase 1's XOR D_b, one table per phase-3 layer b (twiddles are
    // GF(2)-linear in the global group index, so are the perm tables:
    // D_b = the table of group (t_i ^ t_f) * n / 2^(b+1)), kept after the shared tables
#ifdef RS_MONO_ENC_DERIVE3
    static constexpr bool kDerive3 = true;
#else
    static constexpr bool kDerive3 = false;
#endif
    static constexpr uint32_t kD = kDerive3 ? NB3 : 0;
    static constexpr uint32_t words_enc = words + kD * SW;
    static constexpr uint32_t words_dec = words + n;  // + per-row decode info (fused eval_poly)
    // SPLIT decode: + a second column plane (the cross-half step's formal-derivative values)
    static constexpr uint32_t words_split = words_dec + (SPLIT ? plane_words : 0);
    static_assert(L > 11 || (words_enc * 4 <= 160 * 1024 && words_split * 4 <= 160 * 1024), "column kernel: LDS per workgroup");
};

// Table source: tables staged in LDS (STAGED column kernel).  Phase 1 (IFFT
// layers with the low bits in-wave) and phase 3 (FFT layers likewise) read a
// wave-private region: a wave's rows there are 2^IW consecutive rows, so its
// groups are its own.  Phase 2 (top bits in-wave, wave bits low) reads the
// region shared by all waves.
template <int L, int LR, int SPLIT = 0, int E = 4>
struct LdsTabs {
    using G = Stage<L, LR, SPLIT, E>;
    const uint32_t *priv, *shared, *img_i, *img_f;
    template <int, int, typename S, int I, int PH>
    __device__ __forceinline__ void get(int x, uint32_t row, uint32_t (&t)[Fmt<E>::kTW]) const {
#ifdef RS_MONO_FAKE_TABS  // tools/mono_probe.hip: tables without LDS traffic
        const uint32_t *fb = tab<0, 0, S, I, PH>(x, row);
        for (int q = 0; q < G::TW; ++q) t[q] = q + uint32_t(reinterpret_cast<uintptr_t>(fb));
        return;
#endif
        read(tab<0, 0, S, I, PH>(x, row), t);
    }
    static __device__ __forceinline__ void read(const uint32_t *tb, uint32_t (&t)[Fmt<E>::kTW]) {
        const uint4 *p = reinterpret_cast<const uint4 *>(tb);
#pragma unroll
        for (int q = 0; q < int(G::PC); ++q) {
            const uint4 v = p[q];
            t[4 * q] = v.x, t[4 * q + 1] = v.y, t[4 * q + 2] = v.z, t[4 * q + 3] = v.w;
        }
    }
    // the LDS slot of the table of row `row`'s butterfly group at layer x
    template <int, int, typename S, int I, int PH>
    __device__ __forceinline__ const uint32_t *tab(int x, uint32_t row) const {
        uint32_t slot;
        const uint32_t *base;
        if constexpr ((PH == 1 || PH == 3) && G::B0 == 1 && S::v.ops[I].bit == 0) {
            slot = G::sg((row & (G::W - 1)) >> 1);  // layer 0's turn in the region
            base = priv;
        } else if constexpr (PH == 1 || PH == 3) {
            slot = (G::W >> G::B0) - (G::W >> x) + G::sg((row & (G::W - 1)) >> (x + 1));
            base = priv;
        } else if constexpr (PH == 2) {
            slot = (G::n >> G::IW) - (G::n >> x) + G::sg(row >> (x + 1));
            base = shared;
        } else {
            slot = G::kShI + (G::n >> G::FLO) - (G::n >> x) + G::sg(row >> (x + 1));
            base = shared;
        }
        return base + slot * G::SW;
    }
};


// Phase of op I of a sequence: 1 = IFFT in-wave low bits, 2 = IFFT top bits,
// 4 = FFT top bits (shared region, FFT part), 3 = FFT in-wave low bits.
constexpr int remap_index(const Seq &s) {
    for (int i = 0; i < s.count; ++i)
        if (s.ops[i].kind == kOpRemap) return i;
    return s.count;
}
template <typename S, bool FFT, int I>
constexpr int phase_of() {
    constexpr int ri = remap_index(S::v);
    if constexpr (ri == S::v.count) return FFT ? 3 : 1;  // one segment (no wave bits)
    else if constexpr (FFT) return I < ri ? 4 : 3;
    else return I < ri ? 1 : 2;
}

template <int L, int LR, typename S, int I, bool FFT, typename TS, int TW>
__device__ __forceinline__ void load_layer_tabs(const TS &ts, uint32_t lane, uint32_t wave,
                                                uint32_t (&t)[(1 << LR) / 2][TW]) {
    constexpr Op op = S::v.ops[I];
    const uint32_t lr = lane_rows<S, I>(lane, wave);
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (!((i >> op.rs) & 1))
            ts.template get<L, LR, S, I, phase_of<S, FFT, I>()>(op.bit, lr | reg_rows<S, I, LR>(i),
                                                                t[pair_of(i, op.rs)]);
    });
}

template <int L, int LR, typename S, int I, bool IFFT, int E>
__device__ __forceinline__ void apply_layer(const uint32_t (&t)[(1 << LR) / 2][Fmt<E>::kTW], Col<L, LR, E> &c) {
    constexpr Op op = S::v.ops[I];
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int i2 = i | (1 << op.rs);
        if constexpr (!((i >> op.rs) & 1)) {
            if constexpr (E == 2) {
                if constexpr (IFFT) ifft_bfly2(c.lo[i], c.lo[i2], t[pair_of(i, op.rs)]);
                else fft_bfly2(c.lo[i], c.lo[i2], t[pair_of(i, op.rs)]);
            } else {
                if constexpr (IFFT) ifft_bfly(c.lo[i], c.hi[i], c.lo[i2], c.hi[i2], t[pair_of(i, op.rs)]);
                else fft_bfly(c.lo[i], c.hi[i], c.lo[i2], c.hi[i2], t[pair_of(i, op.rs)]);
            }
        }
    });
}

template <int L, int LR, typename S, int I, int E>
__device__ __forceinline__ void apply_xpose(Col<L, LR, E> &c, uint32_t lane) {
    constexpr Op op = S::v.ops[I];
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int i2 = i | (1 << op.rs);
        if constexpr (!((i >> op.rs) & 1)) {
            xpose<op.ls>(c.lo[i], c.lo[i2], lane);
            if constexpr (Fmt<E>::kHi) xpose<op.ls>(c.hi[i], c.hi[i2], lane);
        }
    });
}

// Whole-column exchange through LDS from placement maps[I] to maps[I + 1].
template <int L, int LR, typename S, int I, int E>
__device__ __forceinline__ void apply_remap(Col<L, LR, E> &c, uint32_t *plane, uint32_t lane, uint32_t wave) {
    constexpr uint32_t n = 1u << L;
    __syncthreads();
    const uint32_t a = lane_rows<S, I>(lane, wave);
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t x = swz<L>(a | reg_rows<S, I, LR>(i));
        plane[x] = c.lo[i];
        if constexpr (Fmt<E>::kHi) plane[n + x] = c.hi[i];
    });
    __syncthreads();
    const uint32_t b = lane_rows<S, I + 1>(lane, wave);
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t x = swz<L>(b | reg_rows<S, I + 1, LR>(i));
        c.lo[i] = plane[x];
        if constexpr (Fmt<E>::kHi) c.hi[i] = plane[n + x];
    });
}

// Layer with a zero twiddle (m = 0: engine_naive.rs:64-68 / 96-100 skip the
// multiply, log_m == GF_MODULUS): both butterflies reduce to b ^= a.
template <int L, int LR, typename S, int I, int E>
__device__ __forceinline__ void apply_xor_layer(Col<L, LR, E> &c) {
    constexpr Op op = S::v.ops[I];
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int i2 = i | (1 << op.rs);
        if constexpr (!((i >> op.rs) & 1)) {
            c.lo[i2] ^= c.lo[i];
            if constexpr (Fmt<E>::kHi) c.hi[i2] ^= c.hi[i];
        }
    });
}

constexpr int layer_at(const Seq &s, int k) {
    for (int i = 0; i < s.count; ++i)
        if (s.ops[i].kind == kOpLayer && k-- == 0) return i;
    return s.count;
}
constexpr int num_layers(const Seq &s) { return layer_ordinal(s, s.count); }

// The same tables with every layer's slot address of the lane computed once, up
// front (one pair per lane, LR = 1), and held in VGPRs: the layers then issue
// their ds_read_b128s straight from a register instead of 3-5 VALU of slot
// arithmetic each, and the arithmetic runs while the prologue's loads are in
// flight (RS_MONO_PRE_ADDR=1; 2^11-row kernels keep LdsTabs: at 4 waves per SIMD
// their 20 more VGPRs would not fit).  NI / NF: whether the IFFT / FFT runs.
// Measured slower, so off (profiles/r06q/pre_addr_ab.txt, same output bytes and the
// GPU suite green with it on): the per-layer arithmetic shares terms between the
// layers of a placement, the pinned addresses cannot, and the headline encode issues
// 2.10 M instead of 2.00 M VALU per launch (8.94 -> 9.08-9.10 us, 2^10-row decode
// at 1 % 9.72-9.75 -> 10.04-10.13 us).
#ifndef RS_MONO_PRE_ADDR
#define RS_MONO_PRE_ADDR 0
#endif
template <int L, int LR, int SPLIT, int E, bool NI, bool NF>
struct LdsTabsPre {
    using T = LdsTabs<L, LR, SPLIT, E>;
    using SI = SeqOf<L, LR, false, SPLIT>;
    using SF = SeqOf<L, LR, true, SPLIT>;
    static_assert(LR == 1, "one table per layer and lane");
    static constexpr int KI = NI ? num_layers(SI::v) : 1, KF = NF ? num_layers(SF::v) : 1;
    const uint32_t *lds0;
    uint32_t ai[KI], af[KF];  // byte offsets from lds0, by layer ordinal
    template <typename S, bool FFT, int K>
    __device__ __forceinline__ void fill(const T &ts, uint32_t lane, uint32_t wave, uint32_t (&a)[K]) {
        static_for<0, K>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int I = layer_at(S::v, k);
            a[k] = uint32_t(reinterpret_cast<const char *>(ts.template tab<0, 0, S, I, phase_of<S, FFT, I>()>(
                                S::v.ops[I].bit, lane_rows<S, I>(lane, wave))) -
                            reinterpret_cast<const char *>(lds0));
            asm volatile("" : "+v"(a[k]));  // computed here, kept in a VGPR
        });
    }
    __device__ __forceinline__ LdsTabsPre(const T &ts, const uint32_t *lds, uint32_t lane, uint32_t wave) : lds0(lds) {
        if constexpr (NI) fill<SI, false>(ts, lane, wave, ai);
        if constexpr (NF) fill<SF, true>(ts, lane, wave, af);
    }
    template <int, int, typename S, int I, int PH>
    __device__ __forceinline__ void get(int, uint32_t, uint32_t (&t)[Fmt<E>::kTW]) const {
        constexpr bool F = std::is_same<S, SF>::value;
        static_assert(F ? NF : NI, "the transform's addresses were not computed");
        constexpr int k = layer_ordinal(S::v, I);
        T::read(reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds0) + (F ? af[k] : ai[k])), t);
    }
};

#ifndef RS_MONO_PF
#define RS_MONO_PF 3
#endif
// Layers of twiddle tables in flight ahead of the layer being computed.
constexpr int kMonoPrefetch = RS_MONO_PF;

struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

// Run one transform sequence.  The tables of layer k + B are requested right
// after layer k, into the registers layer k just released, so table latency
// hides behind B - 1 layers of butterflies.  Requests never cross the remap:
// the tables beyond it may not be in place yet (staged kernel).  `pre_remap`
// runs just before the remap.  KHOOK >= 0: hook() runs right before the
// tables of layer ordinal KHOOK are requested (the staged kernel writes a
// wave-private table region there that the layers before it have read).  A
// wave with `pre` false skips the ops before the remap, with `alive` false
// the ops after it.  zero_top: the transform's skew offset is 0 (image 0), so
// the single twiddle of its top layer L-1 is skew[2^(L-1) - 1] = GF_MODULUS
// (tables.rs:285-324: the 16 such entries are skew[2^b - 1]), a multiply-free layer.
template <int L, int LR, bool FFT, int B0, int KHOOK = -1, int SPLIT = 0, typename TS, typename PreRemap,
          int E, typename Hook = NoHook>
__device__ __forceinline__ void run_seq(const TS &ts, Col<L, LR, E> &c, uint32_t *plane, uint32_t lane, uint32_t wave,
                                        const PreRemap &pre_remap, bool alive = true, bool pre = true,
                                        const Hook &hook = Hook{}, bool zero_top = false) {
    using S = SeqOf<L, LR, FFT, SPLIT>;
    constexpr int NT = (1 << LR) / 2;
    constexpr int NL = num_layers(S::v);
    constexpr int RI = remap_index(S::v);
    constexpr int NL1 = layer_ordinal(S::v, RI);  // layers before the remap
    constexpr int B = B0 < NL ? B0 : NL;
    uint32_t tb[B][NT][Fmt<E>::kTW];
    auto request = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if constexpr (k == KHOOK) hook();
        load_layer_tabs<L, LR, S, layer_at(S::v, k), FFT>(ts, lane, wave, tb[k % B]);
    };
    // first tables of a segment [k0, k1) of layer ordinals
    auto prime = [&](auto k0c, auto k1c) {
        constexpr int k0 = decltype(k0c)::value, k1 = decltype(k1c)::value;
        static_for<k0, (k0 + B < k1 ? k0 + B : k1)>(request);
    };
    if (pre) prime(std::integral_constant<int, 0>{}, std::integral_constant<int, NL1>{});
    auto step = [&](auto ic) {
        constexpr int I = decltype(ic)::value;
        constexpr Op op = S::v.ops[I];
        if constexpr (op.kind == kOpXpose) {
#ifndef RS_MONO_SKIP_XPOSE  // tools/mono_probe.hip ablation
            apply_xpose<L, LR, S, I, E>(c, lane);
#endif
        } else if constexpr (op.kind == kOpRemap) {
            pre_remap();
            RS_MSTAMP(FFT ? 8 : 3);
#ifndef RS_MONO_SKIP_REMAP  // tools/mono_probe.hip ablation
            apply_remap<L, LR, S, I, E>(c, plane, lane, wave);
#endif
            RS_MSTAMP(FFT ? 9 : 4);
            if (alive) prime(std::integral_constant<int, NL1>{}, std::integral_constant<int, NL>{});
        } else {
            constexpr int k = layer_ordinal(S::v, I);
#ifndef RS_MONO_SKIP_LAYERS
            if constexpr (op.bit == L - 1 && RS_MONO_ZERO_TOP) {
                if (zero_top) apply_xor_layer<L, LR, S, I, E>(c);
                else apply_layer<L, LR, S, I, !FFT, E>(tb[k % B], c);
            } else {
                apply_layer<L, LR, S, I, !FFT, E>(tb[k % B], c);
            }
#endif
            constexpr int end = k < NL1 ? NL1 : NL;
            if constexpr (k + B < end) {
                request(std::integral_constant<int, k + B>{});
                asm volatile("" ::: "memory");  // keep the request here, ahead of its use
            }
        }
    };
    // pre: run the ops before the remap (a wave whose rows there are all zero
    // skips them: IFFT layers of zero rows give zero rows); alive: after it
    if constexpr (RI < S::v.count) {
        if (pre) static_for<0, RI>(step);
        step(std::integral_constant<int, RI>{});
        if (alive) static_for<RI + 1, S::v.count>(step);
    } else {
        static_for<0, S::v.count>(step);
    }
}

// Decode: does this wave hold, after the FFT's remap, any row of A.dst?
// (there the wave's rows are one block of 2^IW consecutive rows)
template <int L, int LR, int SPLIT = 0>
__device__ __forceinline__ bool wave_stores(const MonoCore &A, uint32_t wave, uint32_t base = 0) {
    using S = SeqOf<L, LR, true, SPLIT>;
    constexpr int I = S::v.count;
    const uint32_t lo = lane_rows<S, I>(0, wave) + base, hi = lo + (1u << (LR + 6));
    return lo < A.dst.row_end && hi > A.dst.row_begin;
}

// Base pointers of this workgroup's stripe (wave-uniform, computed once).
struct StripeBases {
    const uint8_t *src0, *src1;
    uint8_t *dst;
};
__device__ __forceinline__ StripeBases stripe_bases(const MonoCore &A, uint32_t stripe) {
    return {A.src[0].base + uint64_t(stripe) * A.src_bstride[0], A.src[1].base + uint64_t(stripe) * A.src_bstride[1],
            const_cast<uint8_t *>(A.dst.base) + uint64_t(stripe) * A.dst_bstride};
}

// Addresses of a lane's rows r0 + D (D a compile-time row offset): one 64-bit
// multiply per row map for the lane's first row r0, then a uniform step per row
// (row_ptr per row cost ~30 VALU per row load in the headline encode).  The
// base addresses may lie outside a map's rows; row_at tests the range first.
struct RowBase {
    const uint8_t *p[2];
    uint32_t r0;
};
__device__ __forceinline__ const uint8_t *map_base(const RowMap &m, const uint8_t *base, uint32_t r0) {
    return base + int64_t(int32_t(r0 - m.row_begin)) * int64_t(m.stride);
}
__device__ __forceinline__ RowBase row_base(const MonoCore &A, const StripeBases &sb, uint32_t r0) {
    return RowBase{{map_base(A.src[0], sb.src0, r0), map_base(A.src[1], sb.src1, r0)}, r0};
}
template <uint32_t D>
__device__ __forceinline__ const uint8_t *row_at(const MonoCore &A, const RowBase &b) {
    const uint32_t r = b.r0 + D;
    const uint8_t *p = nullptr;
    if (r - A.src[0].row_begin < A.src[0].row_end - A.src[0].row_begin) p = b.p[0] + uint64_t(D) * A.src[0].stride;
    if (A.nsrc > 1 && r - A.src[1].row_begin < A.src[1].row_end - A.src[1].row_begin)
        p = b.p[1] + uint64_t(D) * A.src[1].stride;
    return p;
}

// Row I/O pairs lanes: lanes 2k and 2k+1 read / write the low and the high
// word of the SAME row (one 64-byte block, one cache line) in one
// instruction, so a wave instruction touches 32 lines instead of 64 -- the
// column kernel's row I/O is bound by lines per instruction.  A 2x2 transpose
// (register pair x lane bit 0) converts between that order and the
// placement's (low, high) of a lane's own rows.
template <typename S, int I, int LR>
__device__ __forceinline__ uint32_t paired_row(uint32_t lane, uint32_t wave, int j) {
    return lane_rows<S, I>((lane & ~1u) | uint32_t(j & 1), wave) | reg_rows<S, I, LR>(j >> 1);
}
// paired_row(lane, wave, j) = paired_row(lane, wave, 0) + paired_delta(j): the lane
// bit 0 and register bits are clear in the first row
template <typename S, int I, int LR>
constexpr uint32_t paired_delta(int j) {
    return (uint32_t(j & 1) << S::v.maps[I].lane[0]) + reg_rows<S, I, LR>(j >> 1);
}

// Load transform rows `chunk * n + row` (placement: start of the IFFT) as
// paired words; finish_col completes them.  Missing rows inside the caller's
// matrices are read and discarded by the decode's scaling.  okm bit j: word j
// belongs to a row of the caller's matrices (others read a stand-in row and
// are zeroed by finish_col, not here: a select on the loaded value would make
// the compiler wait for the load right after issuing it)
// (2-element packs: the paired words are the 16-bit low and high halves)
// (AT_FFT: rows in the placement at the start of the FFT -- the end of the IFFT --
// instead: the half-split kernels' work rows, kMonoHalfF)
template <int L, int LR, int SPLIT = 0, int E = 4, int BYTES = -1, bool AT_FFT = false>
__device__ __forceinline__ void issue_col(const MonoCore &A, uint32_t chunk, const PackIO &io, const StripeBases &sb,
                                          uint32_t (&w)[2 << LR], uint32_t &okm, uint32_t lane, uint32_t wave,
                                          bool live = true) {
    using S = SeqOf<L, LR, AT_FFT, SPLIT>;
    const uint32_t base = chunk * (1u << L);
    const uint32_t off = io.lo + ((lane & 1u) ? io.hi_delta : 0u);
    // a row every lane may read (the first source row): lanes without a row of
    // their own load it and discard it, so every wave issues exactly one load
    // per word -- a branch around the loads would make the compiler's vmcnt
    // waits for OLDER loads (the decode's eval_poly inputs) count the loads in
    // it as absent and wait for these rows too
    const uint8_t *any_row = A.src[0].row_end > A.src[0].row_begin ? sb.src0 : sb.src1;
    okm = 0;
    // BYTES >= 0: the caller has branched on io.bytes (byte-wise packs: tails,
    // unaligned matrices) around its whole prologue.  The decode must: a branch
    // per row here joins a path whose bytes were combined as they landed, and
    // at such joins the compiler copies the loaded words into shared registers
    // -- reads that wait for every row load right after it is issued
    const bool bytes = BYTES < 0 ? io.bytes : BYTES != 0;
    PackIO q = io;
    q.bytes = bytes;
    const RowBase rb = row_base(A, sb, paired_row<S, 0, LR>(lane, wave, 0) + base);
    static_for<0, (2 << LR)>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const uint8_t *p = row_at<paired_delta<S, 0, LR>(j)>(A, rb);
        const bool ok = p != nullptr && live;
        const uint8_t *a = (ok ? p : any_row) + off;
        uint32_t v;
        if constexpr (E == 4) v = ld_word(a, q);
        else if (bytes) v = ld_half(a, q);
        else  // the aligned dword holding the 16-bit half (finish_col picks it out: a
              // zero-extending ushort load gets copied through an AND at the first join)
            v = *reinterpret_cast<const uint32_t *>(a - (reinterpret_cast<uintptr_t>(a) & 3u));
        okm |= uint32_t(ok) << j;
#if defined(RS_MONO_SKIP_IO) || defined(RS_MONO_SKIP_LOADS)
        v = (rb.r0 + paired_delta<S, 0, LR>(j)) * 0x9E3779B9u + off;
#endif
        w[j] = v;
    });
}

// Per-row multiply tables gathered by a quad of lanes (2-element format).  A
// gathered table is one 64-byte line per row; a lane fetching its own row's 4
// pieces touches up to 64 lines per wave instruction, and those gathers bound
// the decode's prologue (the texture path resolves about one line per clock).
// Instead lane p of a quad loads piece p of each of the quad's 4 tables (4
// lanes, one line: 16 lines per instruction), and the multiply is split the
// same way: piece p holds the lookups of 2-bit field p (gf_muladd2's d_p and
// c_p), so lane p forms field p's partial product for all 4 rows and a
// reduce-scatter over the quad XORs them into each row's product.
template <int K>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {  // lane 4j + K's value, to the whole quad
    return __builtin_amdgcn_update_dpp(0, int(v), K * 0x55, 0xF, 0xF, false);
}
// t[4k .. 4k + 3] = piece (lane & 3) of table lut[lg of quad lane k]
__device__ __forceinline__ void quad_gather2(const uint32_t *lut, uint32_t lg, uint32_t lane, uint32_t (&t)[16]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(lut) + (lane & 3u);
    static_for<0, 4>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint4 v = q[quad_bcast<k>(lg) * 4u];
        t[4 * k] = v.x, t[4 * k + 1] = v.y, t[4 * k + 2] = v.z, t[4 * k + 3] = v.w;
    });
}
// x * m of this lane's row, t from quad_gather2 (all 4 lanes of the quad take part)
__device__ __forceinline__ uint32_t quad_mul2(uint32_t x, const uint32_t (&t)[16], uint32_t lane) {
    constexpr uint32_t M = 0x03030303u, C = 0x04040000u;
    auto sel = [](uint32_t v) { return __builtin_amdgcn_bitop3_b32(v, M, C, 0xEA); };
    const uint32_t sh = 2u * (lane & 3u);
    uint32_t part[4];
    static_for<0, 4>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t xk = quad_bcast<k>(x);
        const uint32_t xr = __builtin_amdgcn_alignbit(xk, xk, 16);
        const uint64_t s = ((uint64_t(xr) << 32) | xk) >> sh;
        part[k] = __builtin_amdgcn_perm(t[4 * k + 1], t[4 * k], sel(uint32_t(s))) ^
                  __builtin_amdgcn_perm(t[4 * k + 3], t[4 * k + 2], sel(uint32_t(s >> 32)));
    });
    // reduce-scatter: lane p ends with the XOR over the quad of part[p]
    const bool b1 = lane & 2u, b0 = lane & 1u;
    const uint32_t k0 = (b1 ? part[2] : part[0]) ^ xor_lane<1>(b1 ? part[0] : part[2]);
    const uint32_t k1 = (b1 ? part[3] : part[1]) ^ xor_lane<1>(b1 ? part[1] : part[3]);
    return (b0 ? k1 : k0) ^ xor_lane<0>(b0 ? k0 : k1);
}

// Decode scaling (rate_high.rs:213-231): received rows are multiplied by
// exp(log factor), erased rows become zero; rowinfo is indexed by work row.
// scale_issue requests the multiply tables, finish_col applies them
// (2-element packs: quad-gathered, quad_gather2 / quad_mul2).
template <int L, int LR, int E = 4>
struct ScaleTabs {
    uint32_t t[1 << LR][Fmt<E>::kTW];
    uint32_t erased;  // bit i: register i's row is not received
};
#ifndef RS_MONO_NO_QUAD_GATHER  // (A/B: per-lane gathers of whole tables)
constexpr bool kQuadGather = true;
#else
constexpr bool kQuadGather = false;
#endif
template <int L, int LR, int SPLIT = 0, int E = 4>
__device__ __forceinline__ void scale_issue(const MonoCore &A, const uint32_t *rowinfo, ScaleTabs<L, LR, E> &st,
                                            uint32_t lane, uint32_t wave, bool gather = true) {
    constexpr uint32_t PC = Fmt<E>::kPC;
    using S = SeqOf<L, LR, false, SPLIT>;
    const uint32_t a = lane_rows<S, 0>(lane, wave);
    st.erased = 0;
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t f = rowinfo[a | reg_rows<S, 0, LR>(i)];
        uint32_t lg = f & 0xFFFFu;
#ifdef RS_MONO_SKIP_SCALE  // tools/mono_probe.hip ablation: one shared table
        lg = 0;
#endif
        st.erased |= ((f >> 16) & 1u) << i;
        // rows that are not received read one shared table (log 0: one cache
        // line per instruction; finish_col zeroes those rows), so the gathers
        // are unconditional and the waits for the table staging loads issued
        // before them stay exact (see issue_col)
        if (f & 0x10000u) lg = 0;
        if constexpr (E == 2 && kQuadGather) {
            if (gather) quad_gather2(A.lut, lg, lane, st.t[i]);
        } else if (gather) {  // (wave-uniform: a wave with no received row skips them)
            const uint4 *q = reinterpret_cast<const uint4 *>(A.lut) + lg * PC;
#pragma unroll
            for (int v = 0; v < int(PC); ++v) {
                const uint4 x = q[v];
                st.t[i][4 * v] = x.x, st.t[i][4 * v + 1] = x.y, st.t[i][4 * v + 2] = x.z, st.t[i][4 * v + 3] = x.w;
            }
        }
    });
}

template <int L, int LR, bool SCALE, int E>
__device__ __forceinline__ void finish_col(uint32_t (&w)[2 << LR], uint32_t okm, const ScaleTabs<L, LR, E> *st,
                                           Col<L, LR, E> &c, uint32_t lane, const PackIO &io) {
    // 2-element packs: a word holds its 16-bit half in bytes 0-1, or 2-3 when
    // issue_col loaded the aligned dword around a half at offset 2 mod 4
    const uint32_t sel = E == 2 && !io.bytes && (io.lo & 2u) ? 0x07060302u : 0x05040100u;
    constexpr int R = 1 << LR;
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        // rows outside the caller's matrices are zero; a decode's are not
        // received, so the scaling below zeroes them (the words of a lane pair
        // hold one row: its garbage stays in that row)
        if constexpr (!SCALE) {
            w[2 * i] = (okm >> (2 * i)) & 1u ? w[2 * i] : 0u;
            w[2 * i + 1] = (okm >> (2 * i + 1)) & 1u ? w[2 * i + 1] : 0u;
        }
        xpose<0>(w[2 * i], w[2 * i + 1], lane);
        if constexpr (E == 2) {
            c.lo[i] = __builtin_amdgcn_perm(w[2 * i + 1], w[2 * i], sel);
            if constexpr (SCALE) {
#ifndef RS_MONO_SKIP_SCALEMUL  // tools/valu_account.sh ablation: no multiply of received rows
                if constexpr (kQuadGather) c.lo[i] = quad_mul2(c.lo[i], st->t[i], lane);
                else gf_mul2(c.lo[i], st->t[i]);
#endif
                if ((st->erased >> i) & 1u) c.lo[i] = 0;
            }
        } else {
            c.lo[i] = w[2 * i];
            c.hi[i] = w[2 * i + 1];
            if constexpr (SCALE) {
                gf_mul4(c.lo[i], c.hi[i], st->t[i]);
                if ((st->erased >> i) & 1u) c.lo[i] = c.hi[i] = 0;
            }
        }
    });
}

template <int L, int LR, bool SCALE>
__device__ __forceinline__ void load_col(const MonoCore &A, uint32_t chunk, const PackIO &io, const StripeBases &sb,
                                         Col<L, LR> &c, uint32_t lane, uint32_t wave) {
    uint32_t w[2 << LR];
    uint32_t okm;
    issue_col<L, LR>(A, chunk, io, sb, w, okm, lane, wave);
    ScaleTabs<L, LR> st;
    if constexpr (SCALE) scale_issue<L, LR>(A, A.rowinfo, st, lane, wave);
    finish_col<L, LR, SCALE, 4>(w, okm, &st, c, lane, io);
}

// Reveal (decode, rate_high.rs:241-245): the multiply tables exp(65535 - log
// factor) of the lane's rows at the end of the FFT, for erased rows inside
// A.dst (the others read one shared dummy table, log 0: no extra cache lines).
// 2-element packs gather them ahead (reveal_issue, quad-gathered, before the
// FFT's last in-wave phase), so store_col does not wait for them.
template <int LR>
struct RevealTabs {
    uint32_t t[1 << LR][16];
};
template <typename S, int I, int LR>
__device__ __forceinline__ uint32_t reveal_log(const MonoCore &A, const uint32_t *rowinfo, uint32_t r) {
    const uint32_t f = rowinfo[r];
    const bool need = (f & 0x10000u) && r >= A.dst.row_begin && r < A.dst.row_end;
    return need ? 65535u - (f & 0xFFFFu) : 0u;
}
template <int L, int LR, int SPLIT = 0>
__device__ __forceinline__ void reveal_issue(const MonoCore &A, const uint32_t *rowinfo, RevealTabs<LR> &rt,
                                             uint32_t lane, uint32_t wave, uint32_t base = 0) {
    using S = SeqOf<L, LR, true, SPLIT>;
    constexpr int I = S::v.count;
    const uint32_t a = lane_rows<S, I>(lane, wave) + base;
    static_for<0, (1 << LR)>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        quad_gather2(A.lut, reveal_log<S, I, LR>(A, rowinfo, a | reg_rows<S, I, LR>(i)), lane, rt.t[i]);
    });
}

// Store transform rows `chunk * n + row` that fall in A.dst (placement: end
// of the FFT), paired like the loads.  REVEAL (decode): only erased rows,
// multiplied by exp(65535 - log factor) (rate_high.rs:241-245); rt: tables
// from reveal_issue (2-element packs), else gathered here.
// (AT_IFFT: rows in the placement at the end of the IFFT -- the half-split
// kernels' work rows, kMonoHalfI)
template <int L, int LR, bool REVEAL, int SPLIT = 0, int E = 4, bool AT_IFFT = false>
__device__ __forceinline__ void store_col(const MonoCore &A, const uint32_t *rowinfo, uint32_t chunk,
                                          const PackIO &io, const StripeBases &sb, Col<L, LR, E> &c, uint32_t lane,
                                          uint32_t wave, const RevealTabs<LR> *rt = nullptr) {
    using S = SeqOf<L, LR, !AT_IFFT, SPLIT>;
    constexpr uint32_t PC = Fmt<E>::kPC;
    constexpr int I = S::v.count;
    constexpr int R = 1 << LR;
    const uint32_t base = chunk * (1u << L);
    if constexpr (REVEAL) {
        const uint32_t a = lane_rows<S, I>(lane, wave) + base;
        static_for<0, R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr (E == 2) {
                if (rt) {
#ifndef RS_MONO_SKIP_REVEAL  // tools/valu_account.sh ablation: no reveal multiply
                    c.lo[i] = quad_mul2(c.lo[i], rt->t[i], lane);
#endif
                    return;
                }
            }
            const uint32_t r = a | reg_rows<S, I, LR>(i);
            const uint32_t lg = reveal_log<S, I, LR>(A, rowinfo, r);
            uint32_t t[Fmt<E>::kTW];
            const uint4 *q = reinterpret_cast<const uint4 *>(A.lut) + lg * PC;
#pragma unroll
            for (int v = 0; v < int(PC); ++v) {
                const uint4 x = q[v];
                t[4 * v] = x.x, t[4 * v + 1] = x.y, t[4 * v + 2] = x.z, t[4 * v + 3] = x.w;
            }
            if constexpr (E == 2) gf_mul2(c.lo[i], t);
            else gf_mul4(c.lo[i], c.hi[i], t);
        });
    }
    uint32_t w[2 * R];
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (E == 2) {
            w[2 * i] = c.lo[i] & 0xFFFFu;
            w[2 * i + 1] = c.lo[i] >> 16;
        } else {
            w[2 * i] = c.lo[i];
            w[2 * i + 1] = c.hi[i];
        }
        xpose<0>(w[2 * i], w[2 * i + 1], lane);
    });
    const uint32_t off = io.lo + ((lane & 1u) ? io.hi_delta : 0u);
    const uint32_t r0 = paired_row<S, I, LR>(lane, wave, 0) + base;
    uint8_t *const p0 = const_cast<uint8_t *>(map_base(A.dst, sb.dst, r0));  // (see row_at)
    static_for<0, 2 * R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr uint32_t D = paired_delta<S, I, LR>(j);
        const uint32_t r = r0 + D;
        if (r - A.dst.row_begin < A.dst.row_end - A.dst.row_begin) {
            bool keep = true;
            if constexpr (REVEAL) keep = rowinfo[r] & 0x10000u;
#if defined(RS_MONO_SKIP_IO) || defined(RS_MONO_SKIP_STORES)
            keep = w[j] == 0x12345678u;
#endif
            if (keep) {
                uint8_t *p = p0 + uint64_t(D) * A.dst.stride;
                if constexpr (E == 2) st_half(p + off, w[j], io);
#ifndef RS_MONO_NO_NT_STORE  // streaming (non-temporal) row stores: profiles/r02g/ab_nt
                else if (!io.bytes) __builtin_nontemporal_store(w[j], reinterpret_cast<uint32_t *>(p + off));
#endif
                else st_word(p + off, w[j], io);
            }
        }
    });
}

// ---------------------------------------------------------------------------
// Quad encode (kMonoQuadEnc, rs_device.hpp): the 4-element kernel of 2^L "pair
// rows" runs the 2^(L+1)-row encode of a 2-element column pack.  Pair row q's
// pack = [lo(2q, e0) lo(2q, e1) lo(2q+1, e0) lo(2q+1, e1)] + the high bytes
// likewise: rows 2q and 2q + 1 share every twiddle above row bit 0 (the group of
// layer x >= 1 is row >> (x + 1) = q >> x), so layer x of the rows is layer x - 1
// of the pair rows, with the 2^(L+1)-row image's tables of layers >= 1 (the host
// offsets A.img by the layer-0 tables).  Layer 0 -- the butterflies inside a
// pack -- runs before the IFFT and after the FFT (quad_layer0), on 2-element
// tables staged per wave (kQuad0Slot).
constexpr uint32_t kQuad0Slot = 20;  // words per staged layer-0 table (16 used; 80-B slots spread the banks)

// Row loads of the lane's paired words: word j of pair row Q = its plane's
// 16-bit halves of rows 2Q (bits 0-15) and 2Q + 1 (bits 16-31), each read as the
// aligned dword around it (finish_quad picks the half), 2 loads per word.
template <int L, int LR, int PK>
__device__ __forceinline__ void issue_quad(const MonoCore &A, const PackIO &io, const StripeBases &sb,
                                           uint32_t (&w)[4 << LR], uint32_t &okm, uint32_t lane, uint32_t wave) {
    using S = SeqOf<L, LR, false, PK>;
    const uint32_t off = io.lo + ((lane & 1u) ? io.hi_delta : 0u);
    const uint8_t *any_row = A.src[0].row_end > A.src[0].row_begin ? sb.src0 : sb.src1;
    okm = 0;
    const RowBase rb = row_base(A, sb, 2u * paired_row<S, 0, LR>(lane, wave, 0));
    static_for<0, (2 << LR)>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        static_for<0, 2>([&](auto hc) {
            constexpr int h = decltype(hc)::value;
            const uint8_t *p = row_at<2u * paired_delta<S, 0, LR>(j) + uint32_t(h)>(A, rb);
            const bool ok = p != nullptr;
            const uint8_t *a = (ok ? p : any_row) + off;
            uint32_t v;
            if (io.bytes) v = ld_half(a, io);
            else v = *reinterpret_cast<const uint32_t *>(a - (reinterpret_cast<uintptr_t>(a) & 3u));
#if defined(RS_MONO_SKIP_IO) || defined(RS_MONO_SKIP_LOADS)
            v = (rb.r0 + 2u * paired_delta<S, 0, LR>(j) + uint32_t(h)) * 0x9E3779B9u + off;
#endif
            okm |= uint32_t(ok) << (2 * j + h);
            w[2 * j + h] = v;
        });
    });
}
// halves -> pair-row words (rows outside the caller's matrices are zero), then
// the 4-element finish (paired words -> each lane's own pair rows)
template <int L, int LR>
__device__ __forceinline__ void finish_quad(uint32_t (&w)[4 << LR], uint32_t okm, Col<L, LR, 4> &c, uint32_t lane,
                                            const PackIO &io) {
    const uint32_t sel = !io.bytes && (io.lo & 2u) ? 0x07060302u : 0x05040100u;
    uint32_t x[2 << LR];
    static_for<0, (2 << LR)>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const uint32_t h0 = (okm >> (2 * j)) & 1u ? w[2 * j] : 0u, h1 = (okm >> (2 * j + 1)) & 1u ? w[2 * j + 1] : 0u;
        x[j] = io.bytes ? (h0 & 0xFFFFu) | (h1 << 16) : __builtin_amdgcn_perm(h1, h0, sel);
    });
    finish_col<L, LR, false, 4>(x, ~0u, nullptr, c, lane, io);
}
// Stores of the pair rows that fall in A.dst (placement: end of the FFT): each
// word's halves to rows 2Q and 2Q + 1, paired like the loads
template <int L, int LR, int PK>
__device__ __forceinline__ void store_quad(const MonoCore &A, const PackIO &io, const StripeBases &sb,
                                           const Col<L, LR, 4> &c, uint32_t lane, uint32_t wave) {
    using S = SeqOf<L, LR, true, PK>;
    constexpr int I = S::v.count;
    constexpr int R = 1 << LR;
    uint32_t w[2 * R];
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        w[2 * i] = c.lo[i];
        w[2 * i + 1] = c.hi[i];
        xpose<0>(w[2 * i], w[2 * i + 1], lane);
    });
    const uint32_t off = io.lo + ((lane & 1u) ? io.hi_delta : 0u);
    const uint32_t r0 = 2u * paired_row<S, I, LR>(lane, wave, 0);
    uint8_t *const p0 = const_cast<uint8_t *>(map_base(A.dst, sb.dst, r0));  // (see row_at)
    static_for<0, 2 * R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        static_for<0, 2>([&](auto hc) {
            constexpr int h = decltype(hc)::value;
            constexpr uint32_t D = 2u * paired_delta<S, I, LR>(j) + uint32_t(h);
            const uint32_t r = r0 + D;
#if defined(RS_MONO_SKIP_IO) || defined(RS_MONO_SKIP_STORES)
            if (w[j] == 0x12345678u)
#endif
            if (r - A.dst.row_begin < A.dst.row_end - A.dst.row_begin)
                st_half(p0 + uint64_t(D) * A.dst.stride + off, h ? w[j] >> 16 : w[j] & 0xFFFFu, io);
        });
    });
}
// Layer 0 of the rows (engine_naive.rs:96-100 IFFT / :64-68 FFT) on the lane's
// pair rows: a = row 2Q (bytes 0-1 of both planes), b = row 2Q + 1 (bytes 2-3),
// table t of group Q (the 2^(L+1)-row image's layer-0 slot Q, staged at `tabs`)
template <int L, int LR, typename S, int I, bool FFT>
__device__ __forceinline__ void quad_layer0(Col<L, LR, 4> &c, const uint32_t *tabs, uint32_t lane, uint32_t wave) {
    constexpr int R = 1 << LR;
    constexpr uint32_t W = 1u << (LR + 6);
    const uint32_t a0 = lane_rows<S, I>(lane, wave);
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t q = (a0 | reg_rows<S, I, LR>(i)) & (W - 1u);
        uint32_t t[16];
        const uint4 *p = reinterpret_cast<const uint4 *>(tabs + q * kQuad0Slot);
        static_for<0, 4>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const uint4 v = p[k];
            t[4 * k] = v.x, t[4 * k + 1] = v.y, t[4 * k + 2] = v.z, t[4 * k + 3] = v.w;
        });
        // 2-element words [lo0 lo1 hi0 hi1] of the two rows
        uint32_t a = __builtin_amdgcn_perm(c.hi[i], c.lo[i], 0x05040100u);
        uint32_t b = __builtin_amdgcn_perm(c.hi[i], c.lo[i], 0x07060302u);
        if constexpr (FFT) fft_bfly2(a, b, t);
        else ifft_bfly2(a, b, t);
        c.lo[i] = __builtin_amdgcn_perm(b, a, 0x05040100u);
        c.hi[i] = __builtin_amdgcn_perm(b, a, 0x07060302u);
    });
}

// Formal derivative, closed form over the whole column (src/engine/utils.rs:99-104):
//   out[q] = x[q] ^ XOR_{b < L, q_b = 0} x[q | 2^b]   (placement: end of the IFFT)
// Terms on register bits come from the lane's own registers, terms on lane
// bits from the partner lane (DPP / permlane), terms on wave bits through the
// LDS plane -- read only by the waves whose wave bit is clear.
template <int L, int LR, int E>
__device__ __forceinline__ void formal_derivative(Col<L, LR, E> &c, uint32_t *plane, uint32_t lane, uint32_t wave) {
    constexpr bool HI = Fmt<E>::kHi;
    using S = SeqOf<L, LR, true>;
    constexpr uint32_t n = 1u << L;
    constexpr int R = 1 << LR;
    constexpr Map m = S::v.maps[0];
    const uint32_t a = lane_rows<S, 0>(lane, wave);
    constexpr bool kWaves = L > LR + 6;
    if constexpr (kWaves) {
        __syncthreads();  // the plane's previous readers are done
        static_for<0, R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const uint32_t x = swz<L>(a | reg_rows<S, 0, LR>(i));
            plane[x] = c.lo[i];
            if constexpr (HI) plane[n + x] = c.hi[i];
        });
    }
    uint32_t l[R], h[HI ? R : 1];
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        l[i] = c.lo[i];
        if constexpr (HI) h[i] = c.hi[i];
        static_for<0, LR>([&](auto sc) {  // register bits
            constexpr int sb = decltype(sc)::value;
            if constexpr (!((i >> sb) & 1)) {
                l[i] ^= c.lo[i | (1 << sb)];
                if constexpr (HI) h[i] ^= c.hi[i | (1 << sb)];
            }
        });
    });
    static_for<0, 6>([&](auto jc) {  // lane bits
        constexpr int J = decltype(jc)::value;
        const uint32_t keep = (lane >> J) & 1u ? 0u : ~0u;
        static_for<0, R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            l[i] ^= lane_xor<J>(c.lo[i], lane) & keep;
            if constexpr (HI) h[i] ^= lane_xor<J>(c.hi[i], lane) & keep;
        });
    });
    if constexpr (kWaves) {
        __syncthreads();
        static_for<0, 4>([&](auto kc) {  // wave bits (wave-uniform branches)
            constexpr int k = decltype(kc)::value;
            if constexpr (m.wave[k] >= 0) {
                if (!((wave >> k) & 1u)) {
                    static_for<0, R>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        const uint32_t x = swz<L>((a | reg_rows<S, 0, LR>(i)) ^ (1u << m.wave[k]));
                        l[i] ^= plane[x];
                        if constexpr (HI) h[i] ^= plane[n + x];
                    });
                }
            }
        });
    }
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        c.lo[i] = l[i];
        if constexpr (HI) c.hi[i] = h[i];
    });
}

// In-wave terms of the formal derivative (register and lane bits) of the
// values v under placement m: out = v ^ XOR over those bits b with q_b = 0 of
// v[q | 2^b] (src/engine/utils.rs:99-104, closed form).
template <int LR, typename S, bool HI = true>
__device__ __forceinline__ void fd_in_wave(const uint32_t (&vl)[1 << LR], const uint32_t (&vh)[1 << LR],
                                           uint32_t (&l)[1 << LR], uint32_t (&h)[1 << LR], uint32_t lane) {
    constexpr int R = 1 << LR;
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        l[i] = vl[i];
        if constexpr (HI) h[i] = vh[i];
        static_for<0, LR>([&](auto sc) {
            constexpr int sb = decltype(sc)::value;
            if constexpr (!((i >> sb) & 1)) {
                l[i] ^= vl[i | (1 << sb)];
                if constexpr (HI) h[i] ^= vh[i | (1 << sb)];
            }
        });
    });
    static_for<0, 6>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        const uint32_t keep = (lane >> J) & 1u ? 0u : ~0u;
        static_for<0, R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            l[i] ^= lane_xor<J>(vl[i], lane) & keep;
            if constexpr (HI) h[i] ^= lane_xor<J>(vh[i], lane) & keep;
        });
    });
}

// SPLIT decode, the step between the two transforms (placement: end of the
// split IFFT; row bit L-1 = the highest wave bit, the half).  With a = lower-half and
// b = upper-half row of a pair (q, q + n/2):
//   IFFT layer L-1 (engine_naive.rs:96-100):  b' = b ^ a,  a' = a ^ b' * mI
//   formal derivative (closed form): a'' = FD_half(a') ^ b',  b'' = FD_half(b')
//   FFT layer L-1 (engine_naive.rs:64-68):    a3 = a'' ^ b'' * mF,  b3 = b'' ^ a3
// Only the waves of the half `out_half` (the one holding restored rows) go on
// with the FFT; they compute both halves' values of their row positions, so
// the other half's waves only hand over their rows.  Three barriers; every
// wave reaches them.  zi / zf: the IFFT's / FFT's skew offset is 0, so mI / mF
// is zero (run_seq zero_top) and its layer needs no multiply.
template <int L, int LR, int E>
__device__ __forceinline__ void split_top(Col<L, LR, E> &c, uint32_t *plane, uint32_t *plane2, const uint32_t *tab_i,
                                          const uint32_t *tab_f, uint32_t lane, uint32_t wave, uint32_t out_half,
                                          bool zi = false, bool zf = false) {
#ifdef RS_MONO_SKIP_SPLITTOP  // tools/valu_account.sh ablation (every wave skips it: no barrier is left waiting)
    return;
#endif
    zi = zi && RS_MONO_ZERO_TOP;
    zf = zf && RS_MONO_ZERO_TOP;
    using S = SeqOf<L, LR, true, true>;
    constexpr bool HI = Fmt<E>::kHi;
    constexpr int TW = Fmt<E>::kTW;
    constexpr Map m = S::v.maps[0];
    constexpr int KT = L - 1 - (LR + 6);  // the wave bit holding the top row bit (the half)
    static_assert(m.wave[KT] == L - 1, "split placement: the top row bit is the highest wave bit");
    constexpr uint32_t n = 1u << L, H = n >> 1;
    constexpr int R = 1 << LR;
    const uint32_t a = lane_rows<S, 0>(lane, wave);
    const bool out = (wave >> KT) == out_half;
    __syncthreads();  // the plane's previous readers are done
    static_for<0, R>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const uint32_t x = swz<L>(a | reg_rows<S, 0, LR>(i));
        plane[x] = c.lo[i];
        if constexpr (HI) plane[n + x] = c.hi[i];
    });
    __syncthreads();
    uint32_t ll[R], lh[R], ul[R], uh[R];  // lower / upper half values of the lane's row positions
    uint32_t fl[R], fh[R], gl[R], gh[R];  // their in-wave derivative terms (h: E = 4 only)
    uint32_t tf[TW];
    if (out) {
        uint32_t ti[TW];
        static_for<0, TW / 4>([&](auto qc) {  // the top layers' tables: one each, wave-uniform
            constexpr int q = decltype(qc)::value;
            const uint4 v = reinterpret_cast<const uint4 *>(tab_i)[q];
            ti[4 * q] = v.x, ti[4 * q + 1] = v.y, ti[4 * q + 2] = v.z, ti[4 * q + 3] = v.w;
            const uint4 w = reinterpret_cast<const uint4 *>(tab_f)[q];
            tf[4 * q] = w.x, tf[4 * q + 1] = w.y, tf[4 * q + 2] = w.z, tf[4 * q + 3] = w.w;
        });
        static_for<0, R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const uint32_t x = swz<L>((a | reg_rows<S, 0, LR>(i)) ^ H);
            const uint32_t pl = plane[x];
            ll[i] = out_half ? pl : c.lo[i];
            ul[i] = out_half ? c.lo[i] : pl;
            if constexpr (HI) {
                const uint32_t ph = plane[n + x];
                lh[i] = out_half ? ph : c.hi[i];
                uh[i] = out_half ? c.hi[i] : ph;
            }
            if (zi) {
                ul[i] ^= ll[i];
                if constexpr (HI) uh[i] ^= lh[i];
            } else if constexpr (HI) {
                ifft_bfly(ll[i], lh[i], ul[i], uh[i], ti);
            } else {
                ifft_bfly2(ll[i], ul[i], ti);
            }
            // both halves' values, at their own rows, for the wave-bit terms
            const uint32_t y = swz<L>((a | reg_rows<S, 0, LR>(i)) & (H - 1));
            plane2[y] = ll[i];
            plane2[y + H] = ul[i];  // (the upper value of position q sits at swz(q) + H)
            if constexpr (HI) {
                plane2[n + y] = lh[i];
                plane2[n + y + H] = uh[i];
            }
        });
        fd_in_wave<LR, S, HI>(ll, lh, fl, fh, lane);
        fd_in_wave<LR, S, HI>(ul, uh, gl, gh, lane);
    }
    __syncthreads();
    if (out) {
        static_for<0, KT>([&](auto kc) {  // wave bits below the top bit (wave-uniform branches)
            constexpr int k = decltype(kc)::value;
            if constexpr (m.wave[k] >= 0) {
                if (!((wave >> k) & 1u)) {
                    static_for<0, R>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        const uint32_t q = ((a | reg_rows<S, 0, LR>(i)) & (H - 1)) ^ (1u << m.wave[k]);
                        const uint32_t x = swz<L>(q);
                        fl[i] ^= plane2[x];
                        gl[i] ^= plane2[x + H];
                        if constexpr (HI) {
                            fh[i] ^= plane2[n + x];
                            gh[i] ^= plane2[n + x + H];
                        }
                    });
                }
            }
        });
        static_for<0, R>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            fl[i] ^= ul[i];  // bit L-1 term: lower rows take their upper partner (pre-derivative)
            if constexpr (HI) fh[i] ^= uh[i];
            if (zf) {
                gl[i] ^= fl[i];
                if constexpr (HI) gh[i] ^= fh[i];
            } else if constexpr (HI) {
                fft_bfly(fl[i], fh[i], gl[i], gh[i], tf);
            } else {
                fft_bfly2(fl[i], gl[i], tf);
            }
            if constexpr (HI) c.hi[i] = out_half ? gh[i] : fh[i];
            c.lo[i] = out_half ? gl[i] : fl[i];
        });
    }
}

// ---------------------------------------------------------------------------
// eval_poly fused into the staged decode (rs_eval.hip has the standalone
// kernel; same reduction to 2^L points, src/engine/utils.rs:20-31).  Thread t
// holds work rows 2t and 2t+1 (2 rows per lane), so the Walsh-Hadamard layer
// on row bit 0 runs in registers, bits 1..6 across lanes, and the wave bits
// through LDS ping-pong buffers (two bits per barrier).  Mod 65535 throughout.
__device__ __forceinline__ uint32_t ev_add(uint32_t a, uint32_t b) {
    const uint32_t s = a + b;
    return (s + (s >> 16)) & 0xFFFFu;
}

// The transform reduces lazily: values stay below a bound B_k after k layers
// (B_0 = 2^16; a layer maps a < B, b < B to a + b and a - b + M_k, M_k the
// least multiple of 65535 >= B_k, so B_{k+1} = 2 B_k + 65535 < 2^29 for
// k <= 11) and are folded back below 2^16 once at the end.  With the lane's
// role as a mask m (0: lower element, ~0: upper) both outputs are
// partner + (own ^ m) + (m & (M_k + 1)): two VALU per value and layer.
constexpr uint64_t walsh_bound(int k) {
    uint64_t b = 65536u;
    for (int i = 0; i < k; ++i) b = 2 * b + 65535u;
    return b;
}
template <int K>  // M_K + 1 (a template constant: folded at compile time)
constexpr uint32_t kWalshM1 = uint32_t((walsh_bound(K) + 65534u) / 65535u * 65535u) + 1u;
static_assert(walsh_bound(12) < (1ull << 32), "lazy Walsh-Hadamard bound");

__device__ __forceinline__ uint32_t walsh_fold(uint32_t x) {
    x = (x & 0xFFFFu) + (x >> 16);  // < 2^16 + 2^13
    return (x & 0xFFFFu) + (x >> 16);  // < 2^16, same residue mod 65535
}

// rounds of LDS exchanges of one col_walsh (two wave-bit layers per round)
template <int L>
constexpr int kWalshRounds = ((L > 7 ? L - 7 : 0) + 1) / 2;
// G0: index of the transform's first round among the decode's consecutive rounds.
// Round g uses buffer (g even: buf + 2^L words, g odd: buf); the two transforms
// have the same even number of rounds in all, so the last one reads buf and
// every buffer is rewritten only after a barrier that follows its last reads
// (no barrier between the transforms; see col_eval_poly)
template <int L, int G0 = 0, int ST = -1>
__device__ __forceinline__ void col_walsh(uint32_t (&x)[2], uint32_t *buf) {
    const uint32_t t = threadIdx.x, lane = t & 63u;
    {
        const uint32_t p = x[0], q = x[1];
        x[0] = p + q;
        x[1] = p + ~q + kWalshM1<0>;
    }
    static_for<1, (L < 7 ? L : 7)>([&](auto jc) {
        constexpr int k = decltype(jc)::value;  // layer k = row bit k = lane bit k - 1
        constexpr int J = k - 1;
        const uint32_t m = (lane & (1u << J)) ? ~0u : 0u;
        const uint32_t c = m & kWalshM1<k>;
        static_for<0, 2>([&](auto kc) {
            constexpr int q = decltype(kc)::value;
            const uint32_t y = lane_xor<J>(x[q], lane);
            x[q] = y + (x[q] ^ m) + c;
        });
    });
    if constexpr (ST >= 0) RS_MSTAMP(ST);
    // wave bits: two layers per LDS round (each thread reads its group's 3
    // partners), ping-pong buffers so one barrier per round suffices
    static_for<0, ((L > 7 ? L - 7 : 0) + 1) / 2>([&](auto rc) {
        constexpr int rnd = decltype(rc)::value;
        constexpr int j = 7 + 2 * rnd;  // row bits j (and j + 1) = layers j (and j + 1)
        constexpr bool two = j + 1 < L;
        constexpr uint32_t h1 = 1u << (j - 1), h2 = two ? 1u << j : 0u;  // thread bits
        // a thread's two values as one 8-byte word: ds_write_b64 / ds_read_b64 of
        // consecutive threads are conflict-free (stride-2 32-bit accesses were 2-way)
        uint2 *b = reinterpret_cast<uint2 *>(buf + ((((G0 + rnd) & 1) ^ 1) << L));
        b[t] = uint2{x[0], x[1]};
        __syncthreads();
        const uint32_t m1 = (t & h1) ? ~0u : 0u, c1 = m1 & kWalshM1<j>;
        if constexpr (!two) {
            const uint2 y = b[t ^ h1];
            x[0] = y.x + (x[0] ^ m1) + c1;
            x[1] = y.y + (x[1] ^ m1) + c1;
        } else {
            // v[b2][b1] of the group; this thread is (u2, u1)
            const uint32_t m2 = (t & h2) ? ~0u : 0u, c2 = m2 & kWalshM1<j + 1>;
            const uint32_t g0 = t & ~(h1 | h2);
            const uint2 v00 = b[g0], v01 = b[g0 | h1], v10 = b[g0 | h2], v11 = b[g0 | h1 | h2];
            // layer j: own-role element of each pair (v?0 lower, v?1 upper)
            const uint32_t lo0 = v00.x + (v01.x ^ m1) + c1, lo1 = v00.y + (v01.y ^ m1) + c1;
            const uint32_t hi0 = v10.x + (v11.x ^ m1) + c1, hi1 = v10.y + (v11.y ^ m1) + c1;
            x[0] = lo0 + (hi0 ^ m2) + c2;  // layer j + 1
            x[1] = lo1 + (hi1 ^ m2) + c2;
        }
    });
    x[0] = walsh_fold(x[0]);
    x[1] = walsh_fold(x[1]);
}

// eval_poly with two LDS remaps instead of four exchange rounds (L = 10, 3 wave bits;
// RS_MONO_EVAL_REMAP=0: col_walsh's rounds everywhere, 2: also L = 11).  Walsh-Hadamard layers on
// different bits commute, and only the final layout matters (rows 2t, 2t + 1), so:
//   layout O (as col_walsh): point p = k | lane << 1 | wave << 7
//   layout T: bits 7..L-1 on lane bits 0..WB-1 (WB = L - 7 wave bits), bits 1..6-WB on
//             lane bits WB..5, bits 7-WB..6 on the wave bits, bit 0 = k
// transform 1: bits 0..6 in O, remap O -> T, bits 7..L-1; x lw_fold (in T); transform 2:
// bits 7..L-1, 0, 1..6-WB in T, remap T -> O, bits 7-WB..6.  The two remaps use the two
// buffers the rounds used, the last one `buf` (see col_eval_poly on what is written next).
#ifndef RS_MONO_EVAL_REMAP
#define RS_MONO_EVAL_REMAP 1
#endif
// Measured (profiles/r06o/eval_remap_ab.txt, µs per launch, 3 alternating rounds, same output):
// 2^10 work rows 1 % / 100 % 8.84-8.91 / 8.59-8.61 -> 8.68-8.76 / 8.37-8.44; 2^11 1 %
// 12.38-12.54 -> 12.24-12.50 but 100 % 12.24-12.35 -> 12.40-12.54.  So 2^10 only
// (RS_MONO_EVAL_REMAP=2: 2^11 too).
template <int L>
constexpr bool kEvalRemap = (RS_MONO_EVAL_REMAP != 0 && L == 10) || (RS_MONO_EVAL_REMAP == 2 && L == 11);
// layout T: the u32 index (point / 2) of a thread's point pair
template <int L>
__device__ __forceinline__ uint32_t eval_t_pair(uint32_t lane, uint32_t wave) {
    constexpr int WB = L - 7;
    return (lane >> WB) | (wave << (6 - WB)) | ((lane & ((1u << WB) - 1u)) << 6);
}
// LDS slot of a point pair q (< 2^(L-1)): its bits 6.. (the wave in layout O, the lane
// bits 0..WB-1 in layout T) XORed into bits 6-WB..5, so the 64 lanes of a wave hit 64
// different low slot bits in both layouts (uint2 slots: conflict-free ds_*_b64)
template <int L>
__device__ __forceinline__ uint32_t eval_swz(uint32_t q) {
    constexpr int WB = L - 7;
    return q ^ ((q >> 6) << (6 - WB));
}
template <int J, int K>
__device__ __forceinline__ void walsh_lane(uint32_t (&x)[2], uint32_t lane) {
    const uint32_t m = (lane & (1u << J)) ? ~0u : 0u;
    const uint32_t c = m & kWalshM1<K>;
    static_for<0, 2>([&](auto kc) {
        constexpr int q = decltype(kc)::value;
        const uint32_t y = lane_xor<J>(x[q], lane);
        x[q] = y + (x[q] ^ m) + c;
    });
}
template <int K>
__device__ __forceinline__ void walsh_reg(uint32_t (&x)[2]) {
    const uint32_t p = x[0], q = x[1];
    x[0] = p + q;
    x[1] = p + ~q + kWalshM1<K>;
}
// O -> T (to_t) or T -> O through uint2 slots of buf (2^L words)
template <int L, bool TO_T>
__device__ __forceinline__ void eval_remap(uint32_t (&x)[2], uint32_t *buf, uint32_t lane, uint32_t wave) {
    uint2 *b = reinterpret_cast<uint2 *>(buf);
    const uint32_t o = threadIdx.x, t = eval_t_pair<L>(lane, wave);
    b[eval_swz<L>(TO_T ? o : t)] = uint2{x[0], x[1]};
    __syncthreads();
    const uint2 v = b[eval_swz<L>(TO_T ? t : o)];
    x[0] = v.x;
    x[1] = v.y;
}
template <int L>
__device__ __forceinline__ void col_eval_poly_remap(const MonoCore &A, uint32_t ebits, uint32_t rbits,
                                                   const uint32_t &lwv, uint32_t *buf, uint32_t *rinfo) {
    constexpr int WB = L - 7;
    static_assert(WB >= 1 && WB <= 4, "eval_poly remap: 1 to 4 wave bits");
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t i0 = 2 * threadIdx.x;
    uint32_t x[2];
    static_for<0, 2>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t e = (ebits >> k) & 1u, i = i0 + k;
        x[k] = A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e;  // (rate_low.rs:196)
    });
    // transform 1: bits 0..6 (layout O), then bits 7..L-1 (layout T)
    walsh_reg<0>(x);
    static_for<0, 6>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        walsh_lane<J, J + 1>(x, lane);
    });
    RS_MSTAMP(19);
    eval_remap<L, true>(x, buf + (1u << L), lane, wave);
    static_for<0, WB>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        walsh_lane<J, 7 + J>(x, lane);
    });
    x[0] = walsh_fold(x[0]);
    x[1] = walsh_fold(x[1]);
    RS_MSTAMP(14);
    // x lw_fold of the thread's layout-T points (lwv: loaded for that pair, mono_body)
    const uint32_t lw[2] = {lwv & 0xFFFFu, lwv >> 16};
    const bool p0 = lane == 0 && wave == 0;  // layout T's point 0
    static_for<0, 2>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t p = x[k] * lw[k];
        uint32_t f = ev_add(p & 0xFFFFu, p >> 16);
        if (k == 0 && A.low_rate && p0) f = ev_add(f, A.lw0);
        x[k] = f;
    });
    // transform 2: bits 7..L-1, 0, 1..6-WB (layout T), then bits 7-WB..6 (layout O)
    static_for<0, WB>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        walsh_lane<J, J>(x, lane);
    });
    walsh_reg<WB>(x);
    static_for<WB, 6>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        walsh_lane<J, J + 1>(x, lane);
    });
    RS_MSTAMP(20);
    eval_remap<L, false>(x, buf, lane, wave);
    static_for<6 - WB, 6>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        walsh_lane<J, J + WB + 1>(x, lane);
    });
    x[0] = walsh_fold(x[0]);
    x[1] = walsh_fold(x[1]);
    // rinfo of rows 2t, 2t + 1 (layout O), read next by this wave (see col_eval_poly)
    reinterpret_cast<uint2 *>(rinfo)[threadIdx.x] =
        uint2{x[0] | ((rbits & 1u) ? 0u : 0x10000u), x[1] | ((rbits & 2u) ? 0u : 0x10000u)};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// rinfo[r] = log factor | (received ? 0 : 0x10000) for the 2^L work rows.
// ebits / rbits: this thread's erased / received bits (bits 0, 1 = rows 2t,
// 2t+1); lwv: lw_fold of those rows (two 16-bit values), an ordinary load the
// compiler waits for at its first use below, after the first transform -- the
// caller issues it first and calls this on straight-line code after its other
// loads (mono_body), so that wait leaves them in flight.  No barrier at the end
// (see the rinfo store).
template <int L>
__device__ __forceinline__ void col_eval_poly(const MonoCore &A, uint32_t ebits, uint32_t rbits, const uint32_t &lwv,
                                              uint32_t *buf, uint32_t *rinfo) {
    if constexpr (kEvalRemap<L>) {
        col_eval_poly_remap<L>(A, ebits, rbits, lwv, buf, rinfo);
        return;
    }
    const uint32_t i0 = 2 * threadIdx.x;
    uint32_t x[2];
    static_for<0, 2>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t e = (ebits >> k) & 1u, i = i0 + k;
        // high rate: v = e;  low rate: v = e - 1 on [0, end), 0 beyond  (rate_low.rs:196)
        x[k] = A.low_rate ? (i < A.end ? (e ? 0u : 65534u) : 0u) : e;
    });
    col_walsh<L, 0, 19>(x, buf);
    RS_MSTAMP(14);
    const uint32_t lw[2] = {lwv & 0xFFFFu, lwv >> 16};
    static_for<0, 2>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t p = x[k] * lw[k];
        uint32_t f = ev_add(p & 0xFFFFu, p >> 16);
        if (A.low_rate && i0 + k == 0) f = ev_add(f, A.lw0);
        x[k] = f;
    });
    col_walsh<L, kWalshRounds<L>, 20>(x, buf);
    // rinfo of rows 2t, 2t + 1: read next (scale_issue) by the same wave -- the
    // IFFT's first placement gives wave w rows [2^IW w, 2^IW (w + 1)) like this
    // one -- so no barrier: the LDS executes a wave's accesses in order.  The
    // LDS written next (table staging over the second exchange buffer) was last
    // read before the last round's barrier
    reinterpret_cast<uint2 *>(rinfo)[threadIdx.x] =
        uint2{x[0] | ((rbits & 1u) ? 0u : 0x10000u), x[1] | ((rbits & 2u) ? 0u : 0x10000u)};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// LDS staging of the twiddle tables (STAGED kernel): 16-byte pieces q of the
// wave-private region (phase 1 from the IFFT image, phase 3 from the FFT
// image) and of the shared region.
template <int L, int LR, int SPLIT, int E>
__device__ __forceinline__ uint4 priv_piece(const uint32_t *img, uint32_t wave, uint32_t q) {
    using G = Stage<L, LR, SPLIT, E>;
    const uint32_t t = q / G::LPC, piece = q - t * G::LPC;
    const uint32_t y = (G::W >> G::B0) - t;                   // in [1, W >> B0]
    const int b = G::IW - int(32 - __builtin_clz(y - 1));    // IW - ceil(log2 y)
    const uint32_t local = t - ((G::W >> G::B0) - (G::W >> b));
    const uint32_t slot = G::n - (G::n >> b) + wave * (G::W >> (b + 1)) + local;
    return reinterpret_cast<const uint4 *>(img)[slot * G::LPC + piece];
}
// 16-byte piece q of the layer-0 tables of wave `wave`'s phase-1 / -3 rows
// (image slots wave * W/2 .. : contiguous, one coalesced read per wave)
template <int L, int LR, int SPLIT, int E>
__device__ __forceinline__ uint4 l0_piece(const uint32_t *img, uint32_t wave, uint32_t q) {
    using G = Stage<L, LR, SPLIT, E>;
    return reinterpret_cast<const uint4 *>(img)[wave * G::kL0 * G::LPC + q];
}
template <int L, int LR, int SPLIT, int E>
__device__ __forceinline__ const uint4 *shared_piece_ptr(const uint32_t *img_i, const uint32_t *img_f, uint32_t q) {
    using G = Stage<L, LR, SPLIT, E>;
    const uint32_t t = q / G::LPC, piece = q - t * G::LPC;
    const uint32_t slot = t < G::kShI ? G::n - (G::n >> G::IW) + t : G::n - (G::n >> G::FLO) + (t - G::kShI);
    return reinterpret_cast<const uint4 *>(t < G::kShI ? img_i : img_f) + slot * G::LPC + piece;
}
// 16-byte piece q of the D tables (Stage::kD): layer b = q / PC of image t_i ^ t_f, group 0
template <int L, int LR, int SPLIT, int E>
__device__ __forceinline__ const uint4 *d_piece_ptr(const uint32_t *img_d, uint32_t q) {
    using G = Stage<L, LR, SPLIT, E>;
    static_assert(!G::kBasis, "D tables: full-table images");
    const uint32_t b = q / G::PC, piece = q - b * G::PC;
    return reinterpret_cast<const uint4 *>(img_d) + (G::n - (G::n >> b)) * G::PC + piece;
}
// one 16-byte piece as a value (a struct copy `x = *p` becomes a memcpy that
// can keep the destination array in scratch)
__device__ __forceinline__ uint4 ld_piece(const uint4 *p) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = *reinterpret_cast<const v4u *>(p);
    return uint4{v.x, v.y, v.z, v.w};
}
// a staging lane's piece index, clamped into the region's [0, count) (count >= 1)
__device__ __forceinline__ uint32_t clamp_piece(uint32_t q, uint32_t count) { return q < count ? q : count - 1u; }
// layer of table slot t of a wave-private region (phases 1 and 3)
template <int L, int LR, int SPLIT, int E>
__device__ __forceinline__ uint32_t priv_layer(uint32_t t) {
    using G = Stage<L, LR, SPLIT, E>;
    const uint32_t y = (G::W >> G::B0) - t;
    return uint32_t(G::IW - int(32 - __builtin_clz(y - 1)));
}

#ifndef RS_MONO_LDS_PF
#define RS_MONO_LDS_PF 2
#endif

// plan kind of a kernel variant (Plan's SP): bit 0 split, bit 1 FLOW (the
// staged decodes, unless RS_MONO_NO_FLOW)
constexpr int mono_pk(int mode, bool staged, bool split) {
#ifndef RS_MONO_NO_FLOW
#ifndef RS_MONO_ENC_NO_FLOW  // (A/B: the decodes only; encodes measured 8.27 -> 7.90 us with FLOW + fetched phase-3 tables)
    const bool flow = staged;
#else
    const bool flow = staged && mode == kMonoDecode;
#endif
#else
    const bool flow = false;
#endif
    return (split ? 1 : 0) | (flow ? 2 : 0);
}

// Kernel arguments held in SGPRs from the kernel's start: the compiler treats
// argument loads as re-loadable and re-issues them next to later uses (one
// serialized scalar round trip each, a dozen of them ahead of the first row
// load).  All of them are loaded first, then pass through one empty asm that
// makes them values the compiler cannot reload; pointers pass as global
// (address space 1) pointers, so accesses through them stay global_* (not flat).
template <typename T>
using gptr = __attribute__((address_space(1))) T *;
template <typename T>
__device__ __forceinline__ gptr<T> as_global(T *p) {
    return (gptr<T>)p;
}

// the argument struct of a kernel variant (MonoCore unless the staged decode)
template <int MODE, bool STAGED>
using MonoArgT = std::conditional_t<MODE == kMonoDecode && STAGED, MonoArgs, MonoCore>;

template <int L, int LR, int MODE, bool STAGED, bool BATCH, bool SPLIT, int E>
__device__ __forceinline__ void mono_body(const MonoArgT<MODE, STAGED> &K) {
    MonoCore A;  // the scalar arguments; the erasure bitmaps stay in K
    uint32_t ew[4] = {0, 0, 0, 0}, rw[4] = {0, 0, 0, 0};  // staged decode: the wave's bitmap words
    {
        uint32_t packs = K.packs, ppx = K.packs_per_xcd, nsrc = K.nsrc;
        gptr<const uint8_t> b0 = as_global(K.src[0].base), b1 = as_global(K.src[1].base);
        gptr<const uint8_t> bd = as_global(K.dst.base);
        uint64_t st0 = K.src[0].stride, st1 = K.src[1].stride, std_ = K.dst.stride;
        uint32_t rb0 = K.src[0].row_begin, re0 = K.src[0].row_end, rb1 = K.src[1].row_begin, re1 = K.src[1].row_end;
        uint32_t rbd = K.dst.row_begin, red = K.dst.row_end;
        gptr<const uint32_t> img = as_global(K.img), lut = as_global(K.lut);
        gptr<const uint16_t> lwf = as_global(K.lw_fold);
        uint32_t ii = K.ifft_img, fi = K.fft_img, fp = K.fmt.full_packs, th = K.fmt.tail_h, iob = K.fmt.io_bytes;
        uint32_t lowr = K.low_rate, endr = K.end, lw0 = K.lw0, oh = K.out_half;
        uint64_t imw = K.img_words;
        if constexpr (STAGED && MODE == kMonoDecode) {  // this wave's words of the erasure bitmaps
            const uint32_t w4 = 4u * __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            static_for<0, 4>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                ew[i] = K.erased[w4 + i];
                rw[i] = K.received[w4 + i];
            });
        }
        asm volatile("" : "+s"(packs), "+s"(ppx), "+s"(nsrc), "+s"(b0), "+s"(b1), "+s"(bd), "+s"(st0), "+s"(st1),
                     "+s"(std_), "+s"(rb0), "+s"(re0), "+s"(rb1), "+s"(re1), "+s"(rbd), "+s"(red), "+s"(img),
                     "+s"(lut), "+s"(lwf), "+s"(ii), "+s"(fi), "+s"(fp), "+s"(th), "+s"(iob), "+s"(lowr),
                     "+s"(endr), "+s"(lw0), "+s"(oh), "+s"(imw), "+s"(ew[0]), "+s"(ew[1]), "+s"(ew[2]), "+s"(ew[3]),
                     "+s"(rw[0]), "+s"(rw[1]), "+s"(rw[2]), "+s"(rw[3]));
        A.img_words = imw;
        A.packs = packs;
        A.packs_per_xcd = ppx;
        A.nsrc = nsrc;
        A.src[0] = RowMap{(const uint8_t *)b0, st0, rb0, re0};
        A.src[1] = RowMap{(const uint8_t *)b1, st1, rb1, re1};
        A.dst = RowMap{(const uint8_t *)bd, std_, rbd, red};
        A.img = (const uint32_t *)img;
        A.lut = (const uint32_t *)lut;
        A.lw_fold = (const uint16_t *)lwf;
        A.ifft_img = ii;
        A.fft_img = fi;
        A.fmt = ShardFormat{fp, th, iob};
        A.low_rate = lowr;
        A.end = endr;
        A.lw0 = lw0;
        A.out_half = oh;
    }
    A.chunks = K.chunks;
    A.elems = K.elems;
    A.ifft_img_step = K.ifft_img_step;
    A.fft_img_step = K.fft_img_step;
    A.rowinfo = K.rowinfo;
    A.fused_eval = K.fused_eval;
    A.split = K.split;
    A.stripes = K.stripes;
    if constexpr (BATCH) {
        A.src_bstride[0] = K.src_bstride[0];
        A.src_bstride[1] = K.src_bstride[1];
        A.dst_bstride = K.dst_bstride;
    }
    if constexpr (MODE >= kMonoHalfIEnc && MODE <= kMonoHalfFDec) {  // half-split kernels
        A.half0 = K.half0;
        A.zero_halves = K.zero_halves;
        A.top_i = K.top_i;
        A.top_f = K.top_f;
    }
    using C = Col<L, LR, E>;
    // plan kind: split; FLOW for the staged decodes (Plan)
    constexpr int PK = mono_pk(MODE, STAGED, SPLIT);
    using G = Stage<L, LR, PK, E>;
    static_assert(!SPLIT || (STAGED && MODE == kMonoDecode), "split plan: staged decode only");
    static_assert(STAGED || E == 4, "2-element packs: staged kernel only");
    constexpr int R = 1 << LR;
    constexpr uint32_t T = 1u << (L - LR);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t *plane = lds;
    // XCD-aware: workgroup b runs on XCD b % 8, so the packs of one 64-byte
    // block (which share cache lines) go to one XCD's L2.
#ifdef RS_MONO_STAMPS  // entry time, before the first kernel-argument load
    {
        const uint32_t sw = blockIdx.x + blockIdx.y * gridDim.x;
        if (threadIdx.x == blockDim.x - 64 && sw < 4096) g_mono_stamps[sw][7] = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0 && sw < 4096) g_mono_stamps[sw][12] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const uint32_t b = blockIdx.x;
    const uint32_t pk = (b & 7u) * A.packs_per_xcd + (b >> 3);
    if (pk >= A.packs) return;
    const StripeBases sb = BATCH ? stripe_bases(A, blockIdx.y) : StripeBases{A.src[0].base, A.src[1].base,
                                                                             const_cast<uint8_t *>(A.dst.base)};
    // the pack's bytes in the caller's rows (tails: shards.rs:38-74)
    // (quad encode: 2-element column packs, computed as 4-element pair-row packs)
    const PackIO io = E == 4 && MODE != kMonoQuadEnc ? pack_io(A.fmt, pk) : pack_io2(A.fmt, pk);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // half-split modes (kMonoHalf*): this workgroup's half; its transform uses one
    // image for the phase tables (ii = fi: the staged regions serve it alone)
    constexpr bool HALF_I = MODE == kMonoHalfIEnc || MODE == kMonoHalfIDec;
    constexpr bool HALF_F = MODE == kMonoHalfFEnc || MODE == kMonoHalfFDec;
    uint32_t ii = A.ifft_img, fi = A.fft_img, hh = 0;
    if constexpr (HALF_I) {
        hh = A.half0 + blockIdx.y;
        ii += hh * A.ifft_img_step;
        fi = ii;
    } else if constexpr (HALF_F) {
        hh = A.out_half + blockIdx.y;
        fi += hh * A.fft_img_step;
        ii = fi;
    }
    const uint32_t *img_i = A.img + uint64_t(ii) * A.img_words;
    const uint32_t *img_f = A.img + uint64_t(fi) * A.img_words;
    const uint32_t *img_d = A.img + uint64_t(ii ^ fi) * A.img_words;
    C c;
    if constexpr (STAGED) {
      // kBytesIO (staged decodes): the pack's row access form, byte-wise (1: tails,
      // unaligned matrices) or not (0), as a compile-time branch around the whole
      // body -- a join of the two forms' row loads makes the compiler copy the loaded
      // words, and those copies wait for the loads (issue_col); -1: decided per load
      auto staged = [&](auto bytes_c) {
        constexpr int kBytesIO = decltype(bytes_c)::value;
            // one chunk in, one chunk out; every table read comes from LDS (layer
            // 0 of phases 1 / 3 from the image when Stage::B0)
            constexpr bool DEC = MODE == kMonoDecode;
            constexpr bool HSC = MODE == kMonoHalfIDec, HFD = MODE == kMonoHalfFDec;
            constexpr bool QUAD = MODE == kMonoQuadEnc;  // (quad encode: see issue_quad)
            // the half-split kernels' work rows: whole 64-byte blocks
            const PackIO io_w = E == 4 ? pack_io(ShardFormat{}, pk) : pack_io2(ShardFormat{}, pk);
            uint32_t *shared = lds + G::plane_words;
            // encodes fetch phase 3's tables from the FFT image (requested when phase 1
            // ends); RS_MONO_ENC_DERIVE3: derive them in LDS from phase 1's (+ the D
            // tables, Stage::kD) -- measured slower with the FLOW plan (commit 7f40027: probe 8.27 -> 7.90 us
            // per headline launch with fetched tables)
            constexpr bool kDerive3 = !DEC && G::kDerive3;
            constexpr uint32_t kSh = kDerive3 ? G::kShared + G::kD : G::kShared;  // shared tables (+ D)
            uint32_t *priv = shared + kSh * G::SW + wave * G::kPriv * G::SW;
            uint32_t *rinfo = lds + G::words;  // decode with fused eval_poly
            constexpr uint32_t PC = G::PC;  // 16-byte pieces per table
            // image pieces per table: PC, or 2 with basis images (Stage::put builds the tables)
            constexpr uint32_t LPC = G::LPC;
            static_assert(!(G::kBasis && kDerive3), "derived phase-3 tables: full-table images");
            constexpr int KP1 = (LPC * G::kUp + 63) / 64;
            constexpr int KP0 = G::B0 ? (LPC * G::kL0 + 63) / 64 : 1;
            constexpr int KP3 = G::kP3 ? (LPC * G::kP3 + 63) / 64 : 1;  // (guarded by q < LPC * kP3)
            constexpr int KSH = kSh ? (LPC * kSh + T - 1) / T : 1;  // (guarded by q < LPC * kSh)
            RS_MSTAMP(0);
            // decode: does this wave's phase-1 row block (2^IW consecutive rows) hold a
            // received row?  If not its rows are zero through phase 1: it loads no
            // rows and no phase-1 tables, and skips the phase-1 layers
            bool live = true;
            if constexpr (DEC) {
                static_assert(!STAGED || (1u << G::IW) / 32 == 4, "a wave's phase-1 rows: its 4 bitmap words");
                live = (rw[0] | rw[1] | rw[2] | rw[3]) != 0;
            }
            // split decode: does this wave's half go on with the FFT (restored rows)?
            bool out_wave = true;
            if constexpr (SPLIT) out_wave = (wave >> (L - 1 - G::IW)) == A.out_half;
            // Phase 3's tables cover the same wave rows, layers and slots as phase
            // 1's, still in the region when phase 1 ran on real tables (live): the
            // same tables when IFFT and FFT share the skew offset (decodes,
            // rate_high.rs:213-245), else phase 1's XOR D_b (encodes, Stage::kD)
#ifndef RS_MONO_NO_REUSE
            const bool same3 = ii == fi;
            const bool reuse3 = live && (same3 || kDerive3);
#else
            const bool same3 = ii == fi;
            const bool reuse3 = HALF_F;  // (the half FFT has no IFFT: its region is staged for phase 3)
#endif

            // every global read is requested before any of them is waited for.
            // Decodes: eval_poly's inputs first.  Thread t's erased / received bits
            // (rows 2t, 2t + 1) are in word t / 16 of the bitmaps: the wave's 4 words
            // are uniform, i.e. scalar loads of the kernel arguments.  Its lw_fold
            // pair is the first vector load, a plain load the compiler tracks: its
            // wait sits at the first use in col_eval_poly, after the rows and table
            // pieces are issued, and leaves those in flight while eval_poly runs
            // (vmcnt(13) in the headline decode, checked by tests/test_isa.py)
            uint32_t ebits = 0, rbits = 0, lwv = 0;
            if constexpr (DEC) {  // the staged decode always evaluates eval_poly itself
                const uint32_t g = lane >> 4, sh = (2u * lane) & 31u;
                const uint32_t e0 = ew[0], e1 = ew[1], e2 = ew[2], e3 = ew[3], r0 = rw[0], r1 = rw[1], r2 = rw[2], r3 = rw[3];
                ebits = (g == 0 ? e0 : g == 1 ? e1 : g == 2 ? e2 : e3) >> sh;
                rbits = (g == 0 ? r0 : g == 1 ? r1 : g == 2 ? r2 : r3) >> sh;
                // lw_fold of rows 2t, 2t + 1 as one dword (the context keeps every
                // 2^u-entry segment 4-byte aligned, rs_codec.cpp rs_context_create)
                // (RS_MONO_EVAL_REMAP: the pair of the thread's layout-T points, col_eval_poly_remap)
                lwv = reinterpret_cast<const uint32_t *>(A.lw_fold)[kEvalRemap<L> ? eval_t_pair<L>(lane, wave)
                                                                                 : threadIdx.x];
                asm volatile("" ::: "memory");  // issued first, ahead of every other load
            }
            // Decodes: a wave whose phase-1 rows hold no received row (!live) loads
            // no rows, no phase-1 tables and no scale tables (uniform branches: the
            // vector-memory issue rate of the ~330 load instructions of a 2^11-row
            // workgroup bounds the prologue, and 7 of 16 waves are not live at 1 %)
#ifndef RS_MONO_DEC_LOAD_ALL
            const bool skip = DEC && !live;
#else
            const bool skip = false;
#endif
            uint32_t w[2 << LR] = {};
            uint32_t okm = 0;
            auto issue_rows = [&](auto bytes) {
                issue_col<L, LR, PK, E, decltype(bytes)::value>(A, HALF_I ? hh : 0u, io, sb, w, okm, lane, wave, live);
            };
            // kMonoHalfF: the two halves' IFFT rows (work rows, placement at the FFT's start)
            uint32_t w2[2 << LR] = {};
            uint32_t okm2 = 0;
            // quad encode: the rows' 16-bit halves (issue_quad), and layer 0's tables of the
            // wave's 2^IW pair rows for the IFFT (image ii) and the FFT (fi): 2-element
            // tables of the 2^(L+1)-row images (A.lut), staged in the wave's two regions
            uint32_t wq[4 << LR] = {};
            uint32_t okmq = 0;
            constexpr uint32_t QW = 1u << G::IW;                   // pair rows (layer-0 tables) per wave
            constexpr int KQ = QUAD ? int((4 * QW + 63) / 64) : 1;  // 16-byte pieces per lane per transform
            uint4 vq[2][KQ];
            uint32_t *const qtab = lds + G::words_enc + wave * 2u * QW * kQuad0Slot;
            auto issue_quad_tabs = [&]() {
                if constexpr (QUAD) {
                    constexpr uint64_t kImg2 = uint64_t((2u << L) - 1u) * 16u;  // words per 2-element image
                    static_for<0, 2>([&](auto fc) {
                        constexpr int f = decltype(fc)::value;
                        const uint4 *src = reinterpret_cast<const uint4 *>(A.lut + (f ? fi : ii) * kImg2) +
                                           uint64_t(wave) * QW * 4u;
                        static_for<0, KQ>([&](auto kc) {
                            const uint32_t q = lane + 64u * decltype(kc)::value;
                            vq[f][kc] = ld_piece(src + (q < 4 * QW ? q : 4 * QW - 1));
                        });
                    });
                }
            };
            auto write_quad_tabs = [&]() {
                if constexpr (QUAD)
                    static_for<0, 2>([&](auto fc) {
                        constexpr int f = decltype(fc)::value;
                        static_for<0, KQ>([&](auto kc) {
                            const uint32_t q = lane + 64u * decltype(kc)::value;
                            if (q < 4 * QW)
                                reinterpret_cast<uint4 *>(qtab + f * QW * kQuad0Slot + (q >> 2) * kQuad0Slot)[q & 3u] =
                                    vq[f][kc];
                        });
                    });
            };
            // phase-1 tables (a live wave loads all of its region's pieces; lanes past
            // the region's end re-read its last piece and do not write it, so the
            // loads are unconditional); B0: layer 0's go into the region first, the
            // layers above when layer 0 has read them (run_seq's hook)
            uint4 v0[KP0], v1[KP1], vs[KSH];
            auto issue_priv = [&]() {
#ifndef RS_MONO_SKIP_STAGE  // tools/mono_probe.hip ablation
                if constexpr (G::B0)
                    static_for<0, KP0>([&](auto kc) {
                        const uint32_t q = clamp_piece(lane + 64u * decltype(kc)::value, LPC * G::kL0);
                        v0[kc] = l0_piece<L, LR, PK, E>(img_i, wave, live ? q : q % LPC);
                    });
                static_for<0, KP1>([&](auto kc) {
                    const uint32_t q = clamp_piece(lane + 64u * decltype(kc)::value, LPC * G::kUp);
                    v1[kc] = priv_piece<L, LR, PK, E>(img_i, wave, live ? q : q % LPC);
                });
#endif
            };
            // the shared region: every thread of the workgroup loads and writes pieces
            auto issue_shared = [&]() {
#ifndef RS_MONO_SKIP_STAGE
                if constexpr (kSh > 0)
                    static_for<0, KSH>([&](auto kc) {
                        const uint32_t q = clamp_piece(threadIdx.x + T * decltype(kc)::value, LPC * kSh);
                        if constexpr (kSh == G::kShared) {
                            vs[kc] = ld_piece(shared_piece_ptr<L, LR, PK, E>(img_i, img_f, q));
                        } else {
                            const uint4 *src = q < PC * G::kShared ? shared_piece_ptr<L, LR, PK, E>(img_i, img_f, q)
                                                                   : d_piece_ptr<L, LR, PK, E>(img_d, q - PC * G::kShared);
                            vs[kc] = ld_piece(src);
                        }
                    });
#endif
            };
            // Decodes, order of the loads around eval_poly (inputs first, see above).
            // RS_MONO_DEC_ORDER 1: the shared tables, the live waves' rows and phase-1
            // tables, all in flight while eval_poly runs, then the scale gathers;
            // 2: rows, eval_poly, gathers, then the tables; 3: shared tables and rows,
            // eval_poly, gathers, phase-1 tables
#ifndef RS_MONO_DEC_ORDER
#define RS_MONO_DEC_ORDER 1
#endif
            constexpr int kOrder = RS_MONO_DEC_ORDER;
            // 4: the shared tables only, eval_poly, then rows, gathers, phase-1 tables
            constexpr bool kShFirst = kOrder != 2, kPrivFirst = kOrder == 1, kRowsFirst = kOrder != 4;
            const uint32_t *ri = A.rowinfo;
            // eval_poly (decodes): the compiler places the wait for lwv at its first
            // use, counting the loads issued since on the path that reaches it; with
            // the row and table loads behind a branch (skipping waves issue none) a
            // wait after the join would have to assume the fewer loads of the skip
            // path and hold live waves until their rows land -- so each path gets its
            // own copy of eval_poly, on straight-line code after its loads
            auto eval = [&]() {
#ifndef RS_MONO_SKIP_EVAL  // tools/mono_probe.hip ablation
                col_eval_poly<L>(A, ebits, rbits, lwv, plane, rinfo);
#else
                rinfo[2 * threadIdx.x] = ebits & 1u ? 0x10000u : lwv & 0xFFFFu;
                rinfo[2 * threadIdx.x + 1] = ebits & 2u ? 0x10000u : lwv >> 16;
                __syncthreads();
#endif
            };
            using kIO = std::integral_constant<int, kBytesIO>;
            if constexpr (HALF_F) {
                issue_col<L, LR, PK, E, 0, true>(A, 0, io_w, sb, w, okm, lane, wave, !(A.zero_halves & 1u));
                issue_col<L, LR, PK, E, 0, true>(A, 1, io_w, sb, w2, okm2, lane, wave, !(A.zero_halves & 2u));
                issue_priv();
                issue_shared();
            } else if constexpr (!DEC) {
                if constexpr (QUAD) issue_quad<L, LR, PK>(A, io, sb, wq, okmq, lane, wave);
                else issue_rows(kIO{});
                issue_priv();
                issue_shared();
                issue_quad_tabs();
            } else {
                if constexpr (kShFirst) issue_shared();
                RS_MSTAMP(16);
                if (skip) {
                    RS_MSTAMP(18);
                    eval();
                } else {
                    if constexpr (kRowsFirst) issue_rows(kIO{});
                    RS_MSTAMP(17);
                    if constexpr (kPrivFirst) issue_priv();
                    RS_MSTAMP(18);
                    eval();
                }
                ri = rinfo;
                RS_MSTAMP(2);
            }
            ScaleTabs<L, LR, E> st;
            // (decodes) the scale gathers go out as soon as eval_poly is done
            if constexpr (DEC) {
                if constexpr (!kRowsFirst)
                    if (!skip) issue_rows(kIO{});
                scale_issue<L, LR, PK, E>(A, ri, st, lane, wave, !skip);
                if constexpr (!kShFirst) issue_shared();
                if constexpr (!kPrivFirst)
                    if (!skip) issue_priv();
            }
            if constexpr (HSC) scale_issue<L, LR, PK, E>(A, A.rowinfo + (hh << L), st, lane, wave, true);
            RS_MSTAMP(13);
            // the layers' table source (LdsTabsPre: slot addresses computed here, while
            // the loads above are in flight)
            const LdsTabs<L, LR, PK, E> ts_lds{priv, shared, img_i, img_f};
            constexpr bool kPreAddr = RS_MONO_PRE_ADDR && LR == 1 && L <= 10;
            const auto ts = [&]() {
                if constexpr (kPreAddr) return LdsTabsPre<L, LR, PK, E, !HALF_F, !HALF_I>(ts_lds, lds, lane, wave);
                else return ts_lds;
            }();
            auto write1 = [&]() {
#ifndef RS_MONO_SKIP_STAGE
                static_for<0, KP1>([&](auto kc) {
                    const uint32_t q = lane + 64u * decltype(kc)::value;
                    if (q < LPC * G::kUp) G::put(priv, q, v1[kc], [](uint32_t p) { return G::at1(p); });
                });
#endif
            };
#ifndef RS_MONO_SKIP_STAGE
            if (!skip) {  // (a skipping wave's region is written by phase 3's tables before use)
                if constexpr (G::B0 && !HALF_F)
                    static_for<0, KP0>([&](auto kc) {
                        const uint32_t q = lane + 64u * decltype(kc)::value;
                        if (q < LPC * G::kL0) G::put(priv, q, v0[kc], [](uint32_t p) { return G::at0(p); });
                    });
                else
                    write1();
            }
#ifdef RS_MONO_HALF_RACE_PROBE
            // tools/half_race_demo.sh: poison the shared region, then hold back every
            // wave but wave 0 before it writes its shared pieces -- a reader that does
            // not wait for the region's writers sees the poison, deterministically
            if constexpr (HALF_F) {
                for (uint32_t q = threadIdx.x; q < kSh * G::SW / 4; q += T)
                    reinterpret_cast<uint4 *>(shared)[q] = uint4{0xEEEEEEEEu, 0xEEEEEEEEu, 0xEEEEEEEEu, 0xEEEEEEEEu};
                __syncthreads();
                if (wave != 0)
                    for (int k = 0; k < 8; ++k) __builtin_amdgcn_s_sleep(127);
            }
#endif
            static_for<0, KSH>([&](auto kc) {
                const uint32_t q = threadIdx.x + T * decltype(kc)::value;
                if (q < LPC * kSh) G::put(shared, q, vs[kc], [](uint32_t p) { return G::atS(p); });
            });
            write_quad_tabs();  // (wave-private: read back by this wave only)
#endif
            C cb;  // kMonoHalfF: the upper half's rows
            if constexpr (HALF_F) {
                finish_col<L, LR, false>(w, okm, &st, c, lane, io_w);
                finish_col<L, LR, false>(w2, okm2, &st, cb, lane, io_w);
            } else if constexpr (QUAD) {
                finish_quad<L, LR>(wq, okmq, c, lane, io);
                quad_layer0<L, LR, SeqOf<L, LR, false, PK>, 0, false>(c, qtab, lane, wave);  // IFFT layer 0 of the rows
            } else {
                finish_col<L, LR, DEC || HSC>(w, okm, &st, c, lane, io);
            }
            RS_MSTAMP(1);
            // phase-3 tables: requested when phase 1 ends, written over this wave's
            // phase-1 tables when phase 2 ends
            uint4 v3[KP3];
            auto issue3 = [&]() {
                if (reuse3) return;
                if constexpr (G::kP3 > 0)
                static_for<0, KP3>([&](auto kc) {
                    const uint32_t q = lane + 64u * decltype(kc)::value;
                    const uint32_t qc = clamp_piece(q, LPC * G::kP3);
                    v3[kc] = priv_piece<L, LR, PK, E>(img_f, wave, out_wave ? qc : qc % LPC);
                });
            };
            auto write3 = [&]() {
                if (reuse3) {
                    if constexpr (kDerive3) {
                        if (same3) return;
                        uint4 x[KP3];
                        static_for<0, KP3>([&](auto kc) {
                            const uint32_t q = lane + 64u * decltype(kc)::value;
                            if (q < PC * G::kP3) {
                                const uint32_t t = q / PC, piece = q - t * PC;
                                const uint4 v = reinterpret_cast<const uint4 *>(priv)[G::at1(q)];
                                const uint4 d = reinterpret_cast<const uint4 *>(shared)[(G::kShared + priv_layer<L, LR, PK, E>(t)) * G::SPC + piece];
                                x[kc] = uint4{v.x ^ d.x, v.y ^ d.y, v.z ^ d.z, v.w ^ d.w};
                            }
                        });
                        static_for<0, KP3>([&](auto kc) {
                            const uint32_t q = lane + 64u * decltype(kc)::value;
                            if (q < PC * G::kP3) reinterpret_cast<uint4 *>(priv)[G::at1(q)] = x[kc];
                        });
                    }
                    return;
                }
                static_for<0, KP3>([&](auto kc) {
                    const uint32_t q = lane + 64u * decltype(kc)::value;
                    if (q < LPC * G::kP3) G::put(priv, q, v3[kc], [](uint32_t p) { return G::at1(p); });
                });
            };
            // B0: the FFT's layer-0 tables (phase 3's last layer), requested while the
            // FFT's phase 2 runs, take their turn in the region before that layer
            uint4 v4[KP0];
            auto issue4 = [&](bool need) {
                if constexpr (G::B0)
                    static_for<0, KP0>([&](auto kc) {
                        const uint32_t q = lane + 64u * decltype(kc)::value;
                        const uint32_t qc = clamp_piece(q, LPC * G::kL0);
                        v4[kc] = l0_piece<L, LR, PK, E>(img_f, wave, need ? qc : qc % LPC);
                    });
            };
            auto write4 = [&]() {
                if constexpr (G::B0)
                    static_for<0, KP0>([&](auto kc) {
                        const uint32_t q = lane + 64u * decltype(kc)::value;
                        if (q < LPC * G::kL0) G::put(priv, q, v4[kc], [](uint32_t p) { return G::at0(p); });
                    });
            };
            // 2-element decodes: the reveal tables are requested just before the FFT's
            // last remap (with phase 3's table writes), so they land while phase 3 runs
            constexpr bool kPreReveal = (DEC || HFD) && E == 2 && kQuadGather;
            RevealTabs<LR> rt;
            auto pre3 = [&](bool alive) {
                return [&, alive]() {
                    write3();
                    (void)alive;
                    if constexpr (kPreReveal)
                        if (alive) reveal_issue<L, LR, PK>(A, ri, rt, lane, wave, HFD ? hh << L : 0u);
                };
            };
            if constexpr (SPLIT) {
                // the wave's half: the highest wave bit in both placements
                constexpr uint32_t kHalfWords = (G::n / 2) / 32;
                uint32_t half_any = 0;
                const uint32_t h = wave >> (L - 1 - G::IW);
                for (uint32_t k = 0; k < kHalfWords; ++k) half_any |= K.received[h * kHalfWords + k];
                // IFFT: a wave whose rows hold no received row skips phase 1 (its rows
                // stay zero), a half without received rows skips phase 2
                run_seq<L, LR, false, RS_MONO_LDS_PF, G::B0 ? 1 : -1, PK>(ts, c, plane, lane, wave, issue3,
                                                                             half_any != 0, live, write1);
                RS_MSTAMP(5);
                using SF = SeqOf<L, LR, true, PK>;
                constexpr int NLF = num_layers(SF::v);
                const bool out = out_wave;
                const bool alive = out && wave_stores<L, LR, PK>(A, wave);
                constexpr uint32_t kTopI = (G::n >> G::IW) - 2, kTopF = G::kShI + (G::n >> G::FLO) - 2;
                split_top<L, LR>(c, plane, lds + G::words_dec, shared + kTopI * G::SW, shared + kTopF * G::SW, lane, wave,
                                 A.out_half, ii == 0, fi == 0);
                RS_MSTAMP(6);
                issue4(alive);
                // FFT below the top layer: only the half that holds restored rows
                run_seq<L, LR, true, RS_MONO_LDS_PF, G::B0 ? NLF - 1 : -1, PK>(ts, c, plane, lane, wave, pre3(alive),
                                                                                  alive, out, write4);
                if (!alive) return;
            } else if constexpr (HALF_F) {
                static_assert(G::WB > 0, "half FFT: the 2^11-row plan");
                // rate_high.rs:235-237 across the halves (a: lower, b: upper row of a pair):
                // IFFT layer 11 (engine_naive.rs:96-100), the formal derivative (closed
                // form: each half's own terms, plus the upper partner for lower rows;
                // utils.rs:99-104), FFT layer 11 (engine_naive.rs:64-68)
                constexpr int TW = Fmt<E>::kTW;
                uint32_t ti[TW], tf[TW];
                static_for<0, TW / 4>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    const uint4 x = reinterpret_cast<const uint4 *>(A.top_i)[q];
                    const uint4 y = reinterpret_cast<const uint4 *>(A.top_f)[q];
                    ti[4 * q] = x.x, ti[4 * q + 1] = x.y, ti[4 * q + 2] = x.z, ti[4 * q + 3] = x.w;
                    tf[4 * q] = y.x, tf[4 * q + 1] = y.y, tf[4 * q + 2] = y.z, tf[4 * q + 3] = y.w;
                });
                static_for<0, R>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    if constexpr (E == 2) ifft_bfly2(c.lo[i], cb.lo[i], ti);
                    else ifft_bfly(c.lo[i], c.hi[i], cb.lo[i], cb.hi[i], ti);
                });
                if constexpr (HFD) {
                    const C bp = cb;
                    formal_derivative<L, LR>(c, plane, lane, wave);
                    formal_derivative<L, LR>(cb, plane, lane, wave);
                    static_for<0, R>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        c.lo[i] ^= bp.lo[i];
                        if constexpr (E == 4) c.hi[i] ^= bp.hi[i];
                    });
                }
                static_for<0, R>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    if constexpr (E == 2) fft_bfly2(c.lo[i], cb.lo[i], tf);
                    else fft_bfly(c.lo[i], c.hi[i], cb.lo[i], cb.hi[i], tf);
                });
                if (hh & 1u) c = cb;
                // The FFT's first layers (phase 4) read the shared region, which every
                // wave of the workgroup wrote above: wait for all of them.  The decode
                // waits inside formal_derivative; the encode had no barrier between
                // those writes and these reads, so a wave could read another wave's
                // slots before they were written -- what LDS held before (often the
                // same tables, left by the previous launch of this kernel on the CU;
                // not on the first launch in a process) -- the round-5 parity failure
                // of test_half_split_encode_matches_oracle[high-1-2049-64-129]
                // (profiles/r05j/pytest_gpu_multiin_fail.log; r06 demonstration:
                // tools/half_race_demo.sh, profiles/r06a/half_race_demo.txt)
#ifndef RS_MONO_NO_HALF_BARRIER
                if constexpr (!HFD) __syncthreads();
#endif
                RS_MSTAMP(6);
                using SF = SeqOf<L, LR, true, PK>;
                constexpr int NLF = num_layers(SF::v);
                const bool alive = !HFD || wave_stores<L, LR, PK>(A, wave, hh << L);
                issue4(alive);
                run_seq<L, LR, true, RS_MONO_LDS_PF, G::B0 ? NLF - 1 : -1, PK>(ts, c, plane, lane, wave, pre3(alive),
                                                                                alive, true, write4, fi == 0);
                if (!alive) return;
            } else if constexpr (G::WB > 0) {
                run_seq<L, LR, false, RS_MONO_LDS_PF, G::B0 ? 1 : -1, PK>(ts, c, plane, lane, wave, issue3, true, live,
                                                                       write1, ii == 0);
                if constexpr (HALF_I) {  // the half's IFFT rows to the work rows; no FFT here
                    store_col<L, LR, false, PK, E, true>(A, ri, hh, io_w, sb, c, lane, wave);
                    RS_MSTAMP(11);
                    return;
                }
                RS_MSTAMP(5);
                using SF = SeqOf<L, LR, true, PK>;
                constexpr int NLF = num_layers(SF::v);
                const bool alive = !DEC || wave_stores<L, LR, PK>(A, wave);
                issue4(alive);  // (waves that stop early all read one table: no branch around the loads)
                if constexpr (DEC) formal_derivative<L, LR>(c, plane, lane, wave);
                run_seq<L, LR, true, RS_MONO_LDS_PF, G::B0 ? NLF - 1 : -1, PK>(ts, c, plane, lane, wave, pre3(alive), alive,
                                                                            true, write4, fi == 0);
                if (!alive) return;
            } else {
                static_assert(!G::B0, "one-segment plans keep every table in the region");
                run_seq<L, LR, false, RS_MONO_LDS_PF, -1, PK>(ts, c, plane, lane, wave, NoHook{}, true, true, NoHook{},
                                                              ii == 0);
                issue3();
                if constexpr (DEC) formal_derivative<L, LR>(c, plane, lane, wave);
                write3();
                run_seq<L, LR, true, RS_MONO_LDS_PF, -1, PK>(ts, c, plane, lane, wave, NoHook{}, true, true, NoHook{},
                                                             fi == 0);
            }
            RS_MSTAMP(10);
            if constexpr (QUAD) {
                using SQ = SeqOf<L, LR, true, PK>;
                quad_layer0<L, LR, SQ, SQ::v.count, true>(c, qtab + QW * kQuad0Slot, lane, wave);  // FFT layer 0
                store_quad<L, LR, PK>(A, io, sb, c, lane, wave);
            } else {
                store_col<L, LR, DEC || HFD, PK>(A, ri, HALF_F ? hh : 0u, io, sb, c, lane, wave,
                                                 kPreReveal && G::WB > 0 ? &rt : nullptr);
            }
            RS_MSTAMP(11);
      };
      if constexpr (MODE == kMonoDecode) {
          if (io.bytes) staged(std::integral_constant<int, 1>{});
          else staged(std::integral_constant<int, 0>{});
      } else {
          staged(std::integral_constant<int, -1>{});
      }
    } else if constexpr (MODE == kMonoEncodeHigh) {
        // rate_high.rs:44-87: recovery = FFT_0(XOR_c IFFT_{c n + n}(chunk c))
        load_col<L, LR, false>(A, 0, io, sb, c, lane, wave);
        run_seq<L, LR, false, kMonoPrefetch>(GlobalTabs{img_i}, c, plane, lane, wave, NoHook{});
        for (uint32_t ch = 1; ch < A.chunks; ++ch) {
            C t;
            load_col<L, LR, false>(A, ch, io, sb, t, lane, wave);
            run_seq<L, LR, false, kMonoPrefetch>(
                GlobalTabs{img_i + uint64_t(ch) * A.ifft_img_step * A.img_words}, t, plane, lane, wave, NoHook{});
            static_for<0, R>([&](auto ic) {
                c.lo[ic] ^= t.lo[ic];
                c.hi[ic] ^= t.hi[ic];
            });
        }
        run_seq<L, LR, true, kMonoPrefetch>(GlobalTabs{img_f}, c, plane, lane, wave, NoHook{});
        store_col<L, LR, false>(A, A.rowinfo, 0, io, sb, c, lane, wave);
    } else if constexpr (MODE == kMonoEncodeLow) {
        // rate_low.rs:44-87: recovery chunk c = FFT_{c n + n}(IFFT_0(original))
        load_col<L, LR, false>(A, 0, io, sb, c, lane, wave);
        run_seq<L, LR, false, kMonoPrefetch>(GlobalTabs{img_i}, c, plane, lane, wave, NoHook{});
        for (uint32_t ch = 0; ch < A.chunks; ++ch) {
            C t = c;
            run_seq<L, LR, true, kMonoPrefetch>(
                GlobalTabs{img_f + uint64_t(ch) * A.fft_img_step * A.img_words}, t, plane, lane, wave, NoHook{});
            store_col<L, LR, false>(A, A.rowinfo, ch, io, sb, t, lane, wave);
        }
    } else {
        // rate_high.rs:213-245 / rate_low.rs:213-245 after eval_poly
        load_col<L, LR, true>(A, 0, io, sb, c, lane, wave);
        run_seq<L, LR, false, kMonoPrefetch>(GlobalTabs{img_i}, c, plane, lane, wave, NoHook{});
        formal_derivative<L, LR>(c, plane, lane, wave);
        run_seq<L, LR, true, kMonoPrefetch>(GlobalTabs{img_f}, c, plane, lane, wave, NoHook{});
        store_col<L, LR, true>(A, A.rowinfo, 0, io, sb, c, lane, wave);
    }
}

template <int L, int LR, int MODE, bool STAGED, bool BATCH, bool SPLIT, int E>
__global__ void __launch_bounds__(1 << (L - LR)) k_mono(const MonoArgT<MODE, STAGED> A) {
    mono_body<L, LR, MODE, STAGED, BATCH, SPLIT, E>(A);
}
#ifndef RS_MONO_LR10
#define RS_MONO_LR10 1
#endif
#ifndef RS_MONO_NO_STAGE
#define RS_MONO_STAGED_MAX_L 11
#else
#define RS_MONO_STAGED_MAX_L 0
#endif
// log2 rows per lane (2^(L - LR) threads, at most 1024): the staged variant
// keeps 2 rows per lane (L <= 11); the unstaged one at most 512 threads
constexpr bool staged_l(int L) { return L <= RS_MONO_STAGED_MAX_L && (L >= 11 || RS_MONO_LR10 == 1); }
// the split decode plan needs a wave bit below the top bit: 2^(LR + 6 + 2) rows or more
constexpr bool split_l(int L) { return L >= 9 && L <= 11; }
constexpr int mono_lr(int L, bool staged) {
    return staged ? 1 : L <= 10 ? (RS_MONO_LR10 < L - 6 ? RS_MONO_LR10 : L - 6) : L - 9;
}

template <int L, int MODE, bool STAGED, bool BATCH = false, bool SPLIT = false, int E = 4>
hipError_t launch_ls(const MonoArgs &A, hipStream_t s) {
    constexpr int LR = mono_lr(L, STAGED);
    using G = Stage<L, LR, mono_pk(MODE, STAGED, SPLIT), E>;
    size_t lds = STAGED ? size_t(SPLIT ? G::words_split : MODE == kMonoDecode ? G::words_dec : G::words_enc) * 4
                        : size_t(8) << L;
    // 2-element packs exist to spread a launch over more CUs: more than half the
    // CU's LDS keeps the dispatcher from doubling workgroups up on one CU
    if (E == 2 && lds <= 80 * 1024) lds = 84 * 1024;
    static std::atomic<uint64_t> attr_devs{0};  // devices whose attribute is set
    if (lds > 65536) {
        hipError_t e = lds_attr_once(
            attr_devs, reinterpret_cast<const void *>(&k_mono<L, LR, MODE, STAGED, BATCH, SPLIT, E>), int(lds));
        if (e != hipSuccess) return e;
    }
    const uint32_t grid = 8u * A.packs_per_xcd;
    k_mono<L, LR, MODE, STAGED, BATCH, SPLIT, E>
        <<<dim3(grid, BATCH ? A.stripes : 1), 1 << (L - LR), lds, s>>>(static_cast<const MonoArgT<MODE, STAGED> &>(A));
    snprintf(launch_name_buf(), kLaunchNameBytes, "k_mono<%d, %d, %d, %s, %s, %s, %d>", L, LR, MODE,
             STAGED ? "true" : "false", BATCH ? "true" : "false", SPLIT ? "true" : "false", E);
    return hipGetLastError();
}

template <int L, int MODE, int E>
hipError_t launch_staged(const MonoArgs &A, hipStream_t s) {
    if constexpr (MODE == kMonoDecode && split_l(L)) {
        if (A.split) {
            if (A.stripes > 1) return launch_ls<L, MODE, true, true, true, E>(A, s);
            return launch_ls<L, MODE, true, false, true, E>(A, s);
        }
    }
    if (A.stripes > 1) return launch_ls<L, MODE, true, true, false, E>(A, s);
    return launch_ls<L, MODE, true, false, false, E>(A, s);
}

// Staged (LDS tables) variant: single-chunk transforms, 2 rows per lane.
template <int L, int MODE>
hipError_t launch_l(const MonoArgs &A, hipStream_t s) {
    // the staged decode evaluates eval_poly itself; the unstaged one reads rowinfo
    if constexpr (staged_l(L)) {
        if (A.chunks == 1) {  // = mono_staged()
            if (MODE == kMonoDecode && !A.fused_eval) return hipErrorInvalidValue;
            if (A.elems == 2) return launch_staged<L, MODE, 2>(A, s);
            return launch_staged<L, MODE, 4>(A, s);
        }
    }
    if (A.fused_eval || A.stripes > 1 || A.elems != 4) return hipErrorInvalidValue;
    return launch_ls<L, MODE, false>(A, s);
}

// RS_MONO_ONLY_L / RS_MONO_ONLY_MODE (development probes, tools/): build the
// kernels of one transform size / one mode only (compile time)
#ifdef RS_MONO_ONLY_L
#define RS_MONO_HAS_L(l) ((l) == RS_MONO_ONLY_L)
#else
#define RS_MONO_HAS_L(l) true
#endif
#ifdef RS_MONO_ONLY_MODE
#define RS_MONO_HAS_MODE(m) ((m) == RS_MONO_ONLY_MODE)
#else
#define RS_MONO_HAS_MODE(m) true
#endif

template <int MODE>
hipError_t launch_m(int L, const MonoArgs &A, hipStream_t s) {
    if constexpr (!RS_MONO_HAS_MODE(MODE)) return hipErrorNotSupported;
    switch (L) {
        case 7: if constexpr (RS_MONO_HAS_L(7)) return launch_l<7, MODE>(A, s); break;
        case 8: if constexpr (RS_MONO_HAS_L(8)) return launch_l<8, MODE>(A, s); break;
        case 9: if constexpr (RS_MONO_HAS_L(9)) return launch_l<9, MODE>(A, s); break;
        case 10: if constexpr (RS_MONO_HAS_L(10)) return launch_l<10, MODE>(A, s); break;
        case 11: if constexpr (RS_MONO_HAS_L(11)) return launch_l<11, MODE>(A, s); break;
        case 12: if constexpr (RS_MONO_HAS_L(12)) return launch_l<12, MODE>(A, s); break;
        default: break;
    }
    return hipErrorNotSupported;
}

}  // namespace

hipError_t launch_mono_half(int mode, uint32_t halves, const MonoArgs &A, hipStream_t s) {
    if (A.packs == 0 || halves == 0) return hipSuccess;
    if (halves > 2 || A.stripes != 1 || A.chunks != 1) return hipErrorInvalidValue;
    if constexpr (!RS_MONO_HAS_L(11)) {
        return hipErrorNotSupported;
    } else {
        auto go = [&](auto mc, auto ec) -> hipError_t {
            constexpr int MODE = decltype(mc)::value, E = decltype(ec)::value;
            constexpr int L = 11, LR = mono_lr(L, true);
            using G = Stage<L, LR, mono_pk(MODE, true, false), E>;
            size_t lds = size_t(G::words_enc) * 4;
            if (E == 2 && lds <= 80 * 1024) lds = 84 * 1024;
            static std::atomic<uint64_t> attr_devs{0};
            hipError_t e = lds_attr_once(attr_devs, reinterpret_cast<const void *>(&k_mono<L, LR, MODE, true, false, false, E>),
                                         int(lds));
            if (e != hipSuccess) return e;
            k_mono<L, LR, MODE, true, false, false, E>
                <<<dim3(8u * A.packs_per_xcd, halves), 1 << (L - LR), lds, s>>>(static_cast<const MonoCore &>(A));
            snprintf(launch_name_buf(), kLaunchNameBytes, "k_mono<%d, %d, %d, true, false, false, %d>", L, LR, MODE, E);
            return hipGetLastError();
        };
        using I2 = std::integral_constant<int, 2>;
        using I4 = std::integral_constant<int, 4>;
        switch (mode) {
            case kMonoHalfIEnc: return A.elems == 2 ? go(std::integral_constant<int, kMonoHalfIEnc>{}, I2{})
                                                    : go(std::integral_constant<int, kMonoHalfIEnc>{}, I4{});
            case kMonoHalfIDec: return A.elems == 2 ? go(std::integral_constant<int, kMonoHalfIDec>{}, I2{})
                                                    : go(std::integral_constant<int, kMonoHalfIDec>{}, I4{});
            case kMonoHalfFEnc: return A.elems == 2 ? go(std::integral_constant<int, kMonoHalfFEnc>{}, I2{})
                                                    : go(std::integral_constant<int, kMonoHalfFEnc>{}, I4{});
            case kMonoHalfFDec: return A.elems == 2 ? go(std::integral_constant<int, kMonoHalfFDec>{}, I2{})
                                                    : go(std::integral_constant<int, kMonoHalfFDec>{}, I4{});
            default: return hipErrorNotSupported;
        }
    }
}

// Quad encode (kMonoQuadEnc): 2^10 rows as the 4-element kernel of 2^9 pair rows,
// 256 threads.  (2^11 rows would need 8 waves' layer-0 regions: 160 KiB of LDS
// with the kernel's own 90 KiB.)
bool quad_supported(int L) { return L == 10 && RS_MONO_HAS_L(9) && RS_MONO_HAS_MODE(kMonoQuadEnc); }

hipError_t launch_quad(int L, const MonoArgs &A, hipStream_t s) {
    if (A.packs == 0) return hipSuccess;
    if (!quad_supported(L) || A.chunks != 1) return hipErrorInvalidValue;
    if constexpr (!(RS_MONO_HAS_L(9) && RS_MONO_HAS_MODE(kMonoQuadEnc))) {
        return hipErrorNotSupported;
    } else {
        auto go = [&](auto bc) -> hipError_t {
            constexpr bool BATCH = decltype(bc)::value;
            constexpr int LQ = 9, LR = mono_lr(LQ, true), MODE = kMonoQuadEnc;
            using G = Stage<LQ, LR, mono_pk(MODE, true, false), 4>;
            constexpr uint32_t QW = 1u << G::IW;
            const size_t lds = (size_t(G::words_enc) + size_t(G::kWaves) * 2u * QW * kQuad0Slot) * 4u;
            static_assert((size_t(G::words_enc) + size_t(G::kWaves) * 2u * QW * kQuad0Slot) * 4u <= 160u * 1024u,
                          "quad encode: LDS per workgroup");
            static std::atomic<uint64_t> attr_devs{0};
            hipError_t e = lds_attr_once(attr_devs, reinterpret_cast<const void *>(&k_mono<LQ, LR, MODE, true, BATCH, false, 4>),
                                         int(lds));
            if (e != hipSuccess) return e;
            k_mono<LQ, LR, MODE, true, BATCH, false, 4>
                <<<dim3(8u * A.packs_per_xcd, BATCH ? A.stripes : 1), 1 << (LQ - LR), lds, s>>>(static_cast<const MonoCore &>(A));
            snprintf(launch_name_buf(), kLaunchNameBytes, "k_mono<%d, %d, %d, true, %s, false, 4>", LQ, LR, MODE,
                     BATCH ? "true" : "false");
            return hipGetLastError();
        };
        return A.stripes > 1 ? go(std::true_type{}) : go(std::false_type{});
    }
}

bool mono_staged(int L, uint32_t chunks) { return L >= 7 && staged_l(L) && chunks == 1; }
bool mono_split(int L) { return split_l(L) && staged_l(L); }
int mono_rows_log2_per_lane(int L, uint32_t chunks) { return mono_lr(L, mono_staged(L, chunks)); }

hipError_t launch_mono(int mode, int L, const MonoArgs &A, hipStream_t s) {
    if (A.packs == 0) return hipSuccess;
    switch (mode) {
        case kMonoEncodeHigh: return launch_m<kMonoEncodeHigh>(L, A, s);
        case kMonoEncodeLow: return launch_m<kMonoEncodeLow>(L, A, s);
        case kMonoDecode: return launch_m<kMonoDecode>(L, A, s);
        default: return hipErrorNotSupported;
    }
}

}  // namespace rs
