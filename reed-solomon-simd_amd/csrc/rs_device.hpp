// Device-side interface of the MI355X Reed-Solomon engine (host <-> kernels).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>

namespace rs {

// A contiguous range of transform rows backed by a caller buffer:
// transform row r in [row_begin, row_end) lives at base + (r - row_begin) * stride.
struct RowMap {
    const uint8_t *base = nullptr;
    uint64_t stride = 0;
    uint32_t row_begin = 0, row_end = 0;
};

// Byte layout of the caller's shard matrices (src / dst RowMaps; the work
// buffers always use whole 64-byte blocks).  Shards of any even length S:
// S / 64 whole blocks (packs 0 .. full_packs - 1 at the usual offsets), then a
// tail of t = S % 64 bytes holding tail_h = t / 2 low bytes followed by
// tail_h high bytes -- the reference's tail layout (src/engine/shards.rs:38-74,
// src/algorithm.md): tail pack p (elements 4p .. 4p + 3 of the last block) has
// its low bytes at 64 * (full_packs / 8) + 4p, its high bytes tail_h bytes
// further, and min(4, tail_h - 4p) valid elements.  io_bytes: some caller
// matrix is not 4-byte aligned (base or row stride); every caller access then
// goes byte by byte.
struct ShardFormat {
    uint32_t full_packs = 0xFFFFFFFFu;  // default: rows of whole 64-byte blocks
    uint32_t tail_h = 0;
    uint32_t io_bytes = 0;
};

// Offsets of pack pk inside a caller row: low word, high word - low word,
// valid elements, and whether the access must go byte by byte.
struct PackIO {
    uint32_t lo, hi_delta, cnt;
    bool bytes;
};
__host__ __device__ inline PackIO pack_io(const ShardFormat &f, uint32_t pk) {
    if (pk < f.full_packs) return {(pk >> 3) * 64u + (pk & 7u) * 4u, 32u, 4u, f.io_bytes != 0};
    const uint32_t p = pk - f.full_packs, e = 4u * p;
    return {(f.full_packs >> 3) * 64u + e, f.tail_h, f.tail_h > e + 4u ? 4u : f.tail_h - e, true};
}
// 2-element packs (column kernel, E = 2): pack pk holds elements 2pk, 2pk + 1 of
// a block (low bytes at 2 * (pk % 16), high bytes 32 further); tail packs as above
// with 2 elements (shards.rs:38-74).
__host__ __device__ inline PackIO pack_io2(const ShardFormat &f, uint32_t pk) {
    const uint32_t full = f.full_packs == 0xFFFFFFFFu ? 0xFFFFFFFFu : f.full_packs * 2u;
    if (pk < full) return {(pk >> 4) * 64u + (pk & 15u) * 2u, 32u, 2u, f.io_bytes != 0};
    const uint32_t e = 2u * (pk - full);
    return {(full >> 4) * 64u + e, f.tail_h, f.tail_h > e + 2u ? 2u : f.tail_h - e, true};
}
__device__ __forceinline__ uint32_t ld_half(const uint8_t *p, const PackIO &io) {
    if (!io.bytes) return *reinterpret_cast<const uint16_t *>(p);
    uint32_t v = p[0];
    if (io.cnt > 1) v |= uint32_t(p[1]) << 8;
    return v;
}
__device__ __forceinline__ void st_half(uint8_t *p, uint32_t v, const PackIO &io) {
    if (!io.bytes) {
        *reinterpret_cast<uint16_t *>(p) = uint16_t(v);
        return;
    }
    p[0] = uint8_t(v);
    if (io.cnt > 1) p[1] = uint8_t(v >> 8);
}
__device__ __forceinline__ uint32_t ld_word(const uint8_t *p, const PackIO &io) {
    if (!io.bytes) return *reinterpret_cast<const uint32_t *>(p);
    uint32_t v = 0;
#pragma unroll
    for (uint32_t e = 0; e < 4; ++e)
        if (e < io.cnt) v |= uint32_t(p[e]) << (8 * e);
    return v;
}
__device__ __forceinline__ void st_word(uint8_t *p, uint32_t v, const PackIO &io) {
    if (!io.bytes) {
        *reinterpret_cast<uint32_t *>(p) = v;
        return;
    }
#pragma unroll
    for (uint32_t e = 0; e < 4; ++e)
        if (e < io.cnt) p[e] = uint8_t(v >> (8 * e));
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) of kernel `fn` on the
// current device, once per device.  The attribute is per device, and one
// process may drive several GPUs through several rs_contexts (each launcher
// runs with its context's device current), so a process-wide flag would skip
// every device after the first.  `done` is the kernel's own bit set of devices
// (atomic: launchers run on many host threads).
inline hipError_t lds_attr_once(std::atomic<uint64_t> &done, const void *fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = dev >= 0 && dev < 64 ? uint64_t(1) << dev : 0;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// One pass of the multi-pass transform (see DESIGN.md "Pass structure").
//
// A workgroup owns one row SET x one 64-pack column SLICE.  A row set is
// 2^K transform rows whose indices differ only in bits [a, a+K):
//   row(j) = s_lo + (j << a) + (s_hi << (a + K)),  s = set index, j = local row.
// A pack is 4 GF(2^16) elements of one row: 4 low bytes at block offset 4p and
// the matching 4 high bytes at 32 + 4p (reference layout, algorithm.md:18-31).
struct PassArgs {
    uint32_t a = 0;        // stride exponent of the row set
    uint32_t nsets = 1;    // row sets of this launch (n >> K, fewer for a pruned reveal)
    uint32_t set_base = 0; // first row set of this launch (pruned decode reveal passes)
    uint32_t n = 1;        // transform size (rows per chunk)
    uint32_t packs = 0;    // packs per row (shard_bytes / 8)
    uint32_t slices = 0;   // ceil(packs / 64)
    uint32_t grid_chunks = 1;  // chunks spread over gridDim.y
    uint32_t in_chunk0 = 0;    // rows load from chunk 0 whatever the grid's chunk (LowRate: one FFT per output chunk)

    // ---- load: transform row r = row(j) + chunk * n
    RowMap src[2];
    uint32_t nsrc = 0;
    const uint32_t *rowinfo = nullptr;  // decode: bits 0-15 log factor, bit 16 = erased (row is zero)
    uint32_t load_scale = 0;            // scale loaded rows by rowinfo (erased rows load as zero)
    const uint8_t *work_in = nullptr;   // if set, rows come from work_in + r * work_stride
    uint64_t work_stride = 0;
    uint32_t in_chunks = 1;             // in-kernel XOR accumulation over chunks

    // ---- transforms
    uint32_t ifft_delta = 0, ifft_delta_step = 0;
    uint32_t fd_mode = 0;               // 0: none, 1: sum_b P_b over local bits, 2: identity + that
    const uint8_t *xor_in = nullptr;    // after fd: x ^= rows of xor_in (stride work_stride)
    uint32_t fft_delta = 0, fft_delta_step = 0;
    uint32_t out_chunks = 1;            // FFT + store repeated per output chunk

    // ---- store: transform row r = row(j) + chunk * n
    uint8_t *work_out = nullptr;        // if set, every row goes to work_out + r * work_stride
    RowMap dst;                         // else rows in [row_begin, row_end) go to dst
    uint32_t reveal = 0;                // store only erased rows, scaled by exp(65535 - factor)

    const uint32_t *tw = nullptr;       // perm tables indexed by skew index (zero table = no multiply)
    const uint32_t *lut = nullptr;      // perm tables indexed by log factor
    // tw / lut hold 8-word basis tables (rs_codec.cpp basis tables), expanded while staging
    uint32_t tab_basis = 0;
    ShardFormat fmt;                    // byte layout of src / dst (work buffers: whole blocks)

    // ---- 2-level decodes (blk_masks = 1): per block b = row >> blk_shift (b < 256),
    // zero_in bit b: the block's work_in rows are zero (never computed; load as zero);
    // keep_out bit b: the block's work_out rows are read later (others are not stored)
    // blk_uniform = 1: every row set of the launch lies inside one block (the
    // passes below the top level): one scalar test per workgroup, no store mask
    uint32_t blk_masks = 0, blk_shift = 0, blk_uniform = 0;
    uint64_t zero_in[4] = {0, 0, 0, 0};
    uint64_t keep_out[4] = {~0ull, ~0ull, ~0ull, ~0ull};

    // ---- single-pass decodes of at most kPassEvalRows work rows (fused_eval = 1):
    // every workgroup evaluates eval_poly itself (as k_eval_poly, rs_eval.hip)
    // into its LDS row info instead of reading rowinfo -- one launch, not two
    uint32_t fused_eval = 0, ev_low_rate = 0, ev_end = 0, ev_lw0 = 0;
    const uint16_t *ev_lw_fold = nullptr;      // lw_fold for 2^K points
    uint32_t ev_erased[2] = {0, 0}, ev_received[2] = {0, 0};

    // ---- the fused top pass of a multi-pass decode (bfly_prune = 1, K <= 6): its
    // local row j lies in block j (the top level's rows are the 2^K blocks of
    // 2^a rows).  zin_local bit j: block j's IFFT input is zero (zero_in);
    // need_local bit j: block j holds restored rows.  The IFFT skips the butterfly
    // groups whose 2^(b+1) rows are all zero (their outputs stay zero), the FFT
    // those that feed no needed block (their rows are never read: the FFT passes
    // below read only the needed blocks' rows)
    uint32_t bfly_prune = 0;
    uint64_t zin_local = 0, need_local = ~0ull;
};
constexpr uint32_t kPassEvalRows = 64;

enum PassFlags {
    kIfft = 1,
    kFft = 2,
    // derived from PassArgs by launch_pass (compile-time kernel variants):
    kMultiIn = 4,
    kMultiOut = 8,
    kScale = 16,
    kFd = 32,
    kXorIn = 64,
    kReveal = 128,
    kEval = 256,  // fused eval_poly (PassArgs::fused_eval)
    // the IFFT's / FFT's local layer K-1 has a zero twiddle: the pass holds the
    // transform's top bit and its skew offset is 0 for every chunk of the launch
    // (rs_kernels.hip launch_k; the variants that have them)
    kZeroI = 512,
    kZeroF = 1024
};

// Launch one pass on `stream`.  K = log2(rows per set).
hipError_t launch_pass(int K, int flags, const PassArgs &args, hipStream_t stream);

// Name of the kernel the last launch_pass / launch_mono call of this thread
// launched, in rocprofv3's short form ("k_pass<8, 3, 4, 1>"): the profiler's
// records (rs_profile_collect) and the committed PMC summaries share it.
constexpr int kLaunchNameBytes = 96;
char *launch_name_buf();

// Column kernel (DESIGN.md "Column kernel"): one workgroup owns ALL n = 2^L
// transform rows of one pack (4 elements of every row), so a whole encode or
// decode runs without any cross-workgroup exchange.  Twiddles come from
// layer-ordered images: image t (transform skew offset t * n) holds, for
// layer b = 0..L-1 and group g < n / 2^(b+1), the perm table of skew index
// g * 2^(b+1) + 2^b + t * n - 1 at table slot n - n / 2^b + g.
// 2-element staged column kernels (k_mono) stage 8-word basis images and build
// their tables in LDS (rs_mono.hip Stage::kBasis) when 1; the host (rs_codec.cpp
// mono_args) hands them the matching images.  Measured no faster there, so 0;
// k_chunks always uses basis images for 2-element packs.
#ifndef RS_MONO_BASIS
#define RS_MONO_BASIS 0
#endif
// The lane kernel (rs_lane.hip) stages the 8-word basis images of its tables
// when 1 (the host, rs_codec.cpp try_lane, hands it the matching images), the
// 16-word images when 0.
// Column kernels skip the multiply of a top layer whose twiddle is zero (skew
// offset 0: rs_mono.hip run_seq zero_top) when 1.
#ifndef RS_MONO_ZERO_TOP
#define RS_MONO_ZERO_TOP 1
#endif
#ifndef RS_LANE_BASIS
#define RS_LANE_BASIS 1
#endif
enum MonoMode {
    kMonoEncodeHigh = 0,
    kMonoEncodeLow = 1,
    kMonoDecode = 2,
    // half-split transforms of 2^12 rows as two launches of 2^11-row column
    // kernels (L = 11): kMonoHalfI* run the IFFT's layers 0..10 on half
    // half0 + blockIdx.y of the rows (image ifft_img + half * ifft_img_step) and
    // store the half's rows to the work rows (dst); kMonoHalfF* load both halves'
    // work rows, run layer 11 of the IFFT (top_i), the formal derivative (Dec),
    // layer 11 of the FFT (top_f) and the FFT's layers 10..0 on half
    // out_half + blockIdx.y (image fft_img + half * fft_img_step), and store /
    // reveal its rows of dst.  *Dec: the decode's scaling (rowinfo) and reveal.
    kMonoHalfIEnc = 3,
    kMonoHalfIDec = 4,
    kMonoHalfFEnc = 5,
    kMonoHalfFDec = 6,
    // quad encode (launch_quad): a single-chunk encode of 2^L rows in 2-element
    // column packs run as the 4-element kernel of 2^(L-1) "pair rows": a pack is
    // 2 elements x rows (2q, 2q + 1), so every layer above row bit 0 multiplies 4
    // elements per table (gf_muladd4, 26 VALU) where the 2-element kernel spends
    // 2 x 24 on them; layer 0 (inside the pack) runs first / last on its own.
    kMonoQuadEnc = 7,
};
constexpr uint32_t kMonoFusedRows = 2048;  // largest work size of the fused-eval_poly decode
// The kernel arguments of every column kernel; the staged decode's kernels take
// MonoArgs (+ the erasure bitmaps), the others this core only: argument bytes
// cost launch time (≈0.4 us per KiB back to back, tools/kernarg_probe.hip).
struct MonoCore {
    uint32_t packs = 0;          // packs per row (shard_bytes / (2 * elems), rounded up)
    uint32_t packs_per_xcd = 0;  // ceil(packs / 8): workgroup b runs pack (b % 8) * packs_per_xcd + b / 8
    RowMap src[2];               // transform rows to load (others are zero)
    uint32_t nsrc = 0;
    RowMap dst;                  // transform rows to store (decode: erased originals only)
    uint32_t chunks = 1;         // high: IFFT chunks XOR-folded; low: FFT output chunks
    const uint32_t *img = nullptr;  // twiddle images of this L, image t at img + t * img_words
    uint64_t img_words = 0;         // (n - 1) * table words (20, or 16 in the 2-element format)
    uint32_t elems = 4;             // pack format: 4 or 2 elements per pack (rs_mono.hip Fmt)
    uint32_t ifft_img = 0, ifft_img_step = 0;  // image of IFFT chunk c: ifft_img + c * ifft_img_step
    uint32_t fft_img = 0, fft_img_step = 0;
    const uint32_t *rowinfo = nullptr;  // decode: bits 0-15 log factor, bit 16 erased
    const uint32_t *lut = nullptr;      // perm tables by log factor (Engine::mul semantics; format of elems)
    // decode with eval_poly fused into the staged kernel (every workgroup
    // evaluates it; no rowinfo; MonoArgs::erased / received)
    uint32_t fused_eval = 0, low_rate = 0, end = 0, lw0 = 0;
    // split plan (mono_split(L)): every restored row lies in half out_half of the 2^L work rows
    uint32_t split = 0, out_half = 0;
    ShardFormat fmt;  // byte layout of src / dst
    const uint16_t *lw_fold = nullptr;
    // a batch of stripes of one shape in one launch (staged kernel, grid.y =
    // stripes): stripe b's rows sit b * *_bstride bytes after the base
    // pointers (read only by the batch instantiation)
    uint32_t stripes = 1;
    uint64_t src_bstride[2] = {0, 0}, dst_bstride = 0;
    // half-split kernels (kMonoHalf*): first half of the launch, halves whose work
    // rows are all zero (bit h; not read), layer-11 perm tables of the IFFT / FFT
    uint32_t half0 = 0, zero_halves = 0;
    const uint32_t *top_i = nullptr, *top_f = nullptr;
};
struct MonoArgs : MonoCore {
    // fused-eval_poly decode: erased / received bits of the 2^L work rows, as in EvalArgs
    uint32_t erased[kMonoFusedRows / 32] = {}, received[kMonoFusedRows / 32] = {};
};
// hipErrorNotSupported: no column kernel for this L (7 <= L <= 12 are built).
hipError_t launch_mono(int mode, int L, const MonoArgs &A, hipStream_t stream);
// Multi-chunk encodes of 2^L rows, 2 <= L <= 7 (rs_chunks.hip): HighRate (high:
// A.chunks input chunks, images ifft_img + c * ifft_img_step, fft_img) or
// LowRate (A.chunks output chunks, images ifft_img, fft_img + c * fft_img_step);
// src[0] / dst, one stripe, A.chunks >= 2, elems 2 or 4.
bool chunks_supported(int L);
// pw: packs per wave (1, 2, 4): each wave transforms its chunks for pw packs
// with one staging of the chunk's tables (A.packs_per_xcd is recomputed).
hipError_t launch_chunks(int L, bool high, const MonoCore &A, hipStream_t stream, int pw = 1);
// kMonoHalf* modes: L = 11 only, one stripe, grid.y = halves (launch_mono_half).
hipError_t launch_mono_half(int mode, uint32_t halves, const MonoArgs &A, hipStream_t stream);
// Quad encode of 2^L rows (kMonoQuadEnc; quad_supported(L)): packs / fmt / rows of
// the 2-element format; img = the 4-element images of 2^L rows offset by 2^(L-1)
// tables (layer 0 skipped), img_words = (2^L - 1) * 20; lut = the 2-element images
// of 2^L rows (their layer-0 tables); one chunk; stripes for a batch.
bool quad_supported(int L);
hipError_t launch_quad(int L, const MonoArgs &A, hipStream_t stream);
// Variant launch_mono picks: LDS-staged twiddles (single chunk, 2 rows per
// lane, L <= 11); fused_eval and stripes > 1 require it.
bool mono_staged(int L, uint32_t chunks);
// Decodes of 2^L work rows (L in 9..11) whose restored rows all lie in one half
// may use the split plan (MonoArgs::split): the FFT below the top layer runs
// only on that half.
bool mono_split(int L);
int mono_rows_log2_per_lane(int L, uint32_t chunks);

// Lane column kernel (rs_lane.hip): the single-chunk encode of 2^L rows
// (lane_supported(L): 8 <= L <= 10) in 2-element packs with one row per thread;
// takes the column kernel's arguments (elems = 2, chunks = 1; stripes for a batch).
bool lane_supported(int L);
hipError_t launch_lane(int L, const MonoCore &A, hipStream_t stream);

// eval_poly for a decode (src/engine/utils.rs:20-31) reduced to 2^u points
// (DESIGN.md "eval_poly"): erasure vector -> per-row log factors.
//   row r < 2^u: erased bit e(r) (erasure-vector entry) and received bit.
//   low_rate: the erasure vector is also 1 on [2^u, 65536) (rate_low.rs:196).
//   end: recovery_end / original_end.
// Output rowinfo[r] = log factor | (received ? 0 : 0x10000).
// Rows' bits travel in the kernel arguments when 2^u <= kEvalInlineRows (no
// copy, no extra launch), else in a device byte array (bit0 erased, bit1 received).
constexpr uint32_t kEvalInlineRows = 8192;
struct EvalArgs {
    uint32_t u = 0, low_rate = 0, end = 0, lw0 = 0;
    const uint16_t *lw_fold = nullptr;  // lw_fold for this u (2^u entries)
    uint32_t *rowinfo = nullptr;
    const uint8_t *state = nullptr;     // 2^u > kEvalInlineRows only
    uint32_t erased[kEvalInlineRows / 32] = {};
    uint32_t received[kEvalInlineRows / 32] = {};
};
hipError_t launch_eval_poly(const EvalArgs &A, hipStream_t stream);

// x[rows] *= exp(log_m) over `blocks` 64-byte blocks.
hipError_t launch_mul(uint8_t *rows, uint64_t blocks, const uint32_t *lut_entry, hipStream_t stream);

// out[q] = in[q] ^ XOR_{b: q_b = 0, 2^b < rows} in[q | 2^b]  (formal derivative, closed form)
hipError_t launch_formal_derivative(const uint8_t *in, uint8_t *out, uint32_t rows, uint64_t row_bytes,
                                    hipStream_t stream);

}  // namespace rs
