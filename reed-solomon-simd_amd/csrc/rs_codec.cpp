// Host side of the MI355X Reed-Solomon engine: GF tables on the device, the
// HighRate / LowRate orchestration as device passes, the encoder / decoder
// objects and the extern "C" boundary declared in include/rs_mi355x.h.
//
// Rate semantics follow reference src/rate/rate_high.rs:44-254,
// src/rate/rate_low.rs:44-254, src/rate/rate_default.rs:15-64; validation and
// error order follow src/rate.rs:91-106, src/rate/encoder_work.rs:50-87,
// src/rate/decoder_work.rs:62-141, src/lib.rs:251-353.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <initializer_list>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../include/rs_mi355x.h"
#include "gf_tables.hpp"
#include "rs_device.hpp"

namespace {

thread_local std::string g_last_error;

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
uint32_t ilog2(uint64_t x) {
    uint32_t l = 0;
    while ((uint64_t(1) << l) < x) ++l;
    return l;
}
uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

struct DevError {
    hipError_t e;
};
void check(hipError_t e) {
    if (e != hipSuccess) throw DevError{e};
}

rs_status set_err(rs_error *err, rs_status code) {
    if (err) {
        std::memset(err, 0, sizeof *err);
        err->code = code;
    }
    return code;
}

// ---------------------------------------------------------------------------
// rate selection (rate_default.rs:15-64, rate_high.rs:19-25, rate_low.rs:19-25)

bool high_supported(uint64_t N, uint64_t M) {
    return N > 0 && M > 0 && N < 65536 && M < 65536 && next_pow2(M) + N <= 65536;
}
bool low_supported(uint64_t N, uint64_t M) {
    return N > 0 && M > 0 && N < 65536 && M < 65536 && next_pow2(N) + M <= 65536;
}
int use_high_rate(uint64_t N, uint64_t M) {
    if (N > 65536 || M > 65536 || N == 0 || M == 0) return -1;
    const uint64_t pn = next_pow2(N), pm = next_pow2(M);
    if (std::min(pn, pm) + std::max(N, M) > 65536) return -1;
    if (pn != pm) return pn > pm ? 1 : 0;
    return N <= M ? 1 : 0;
}

// resolves `rate` for (N, M, S) with the reference's error order; returns
// 1 = high, 0 = low, or sets err and returns -1
int resolve(rs_rate rate, uint64_t N, uint64_t M, uint64_t S, rs_error *err) {
    int high;
    if (rate == RS_RATE_HIGH) high = 1;
    else if (rate == RS_RATE_LOW) high = 0;
    else high = use_high_rate(N, M);
    if (high < 0 || (high ? !high_supported(N, M) : !low_supported(N, M))) {
        set_err(err, RS_ERR_UNSUPPORTED_SHARD_COUNT);
        if (err) err->original_count = N, err->recovery_count = M;
        return -1;
    }
    if (S == 0 || (S & 1)) {
        set_err(err, RS_ERR_INVALID_SHARD_SIZE);
        if (err) err->shard_bytes = S;
        return -1;
    }
    return high;
}

// Device-side scratch that grows monotonically.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    void swap(DevBuf &o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
    }
    void *get(size_t bytes) {
        if (bytes > cap) {
            if (p) check(hipFree(p));
            p = nullptr;
            check(hipMalloc(&p, bytes));
            cap = bytes;
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Pinned host staging that grows monotonically; `ready` orders its reuse
// after the asynchronous copy that last read it.
struct PinnedBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipEvent_t ready = nullptr;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf &operator=(const PinnedBuf &) = delete;
    void swap(PinnedBuf &o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
        std::swap(ready, o.ready);
    }
    uint8_t *get(size_t bytes) {
        if (ready) check(hipEventSynchronize(ready));  // the previous copy out of it is done
        if (bytes > cap) {
            if (p) check(hipHostFree(p));
            p = nullptr;
            check(hipHostMalloc(&p, bytes, hipHostMallocDefault));
            cap = bytes;
        }
        return static_cast<uint8_t *>(p);
    }
    void copied_on(hipStream_t s) {
        if (!ready) check(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        check(hipEventRecord(ready, s));
    }
    ~PinnedBuf() {
        if (ready) (void)hipEventSynchronize(ready), (void)hipEventDestroy(ready);
        if (p) (void)hipHostFree(p);
    }
};

// Device scratch of one stream's calls.  Calls on one stream execute in order,
// so one workspace per (context, stream) makes concurrent calls on different
// streams safe (rs_mi355x.h "Threading and streams").
struct Workspace {
    DevBuf buf[4], rowinfo, state;
    std::vector<uint8_t> h_state;
    PinnedBuf h_state_pinned;  // source of the erasure-state copy of large decodes
    void swap(Workspace &o) {
        for (int k = 0; k < 4; ++k) buf[k].swap(o.buf[k]);
        rowinfo.swap(o.rowinfo);
        state.swap(o.state);
        h_state.swap(o.h_state);
        h_state_pinned.swap(o.h_state_pinned);
    }
};

// Runs the calling thread on `device` for the scope and restores the thread's
// previous current device afterwards (the caller's -- e.g. torch's -- device
// selection is left as it was).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int device) {
        check(hipGetDevice(&prev));
        if (prev != device) check(hipSetDevice(device));
        else prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// Host copies of the one-shot calls (rs_encode / rs_decode, lib.rs:251-353) on a few
// helper threads: the caller's shards into the pinned staging and the recovery rows
// out of it are ~1 MiB memcpy each at the headline shape, ~34 us on one core -- the
// whole difference between the one-shot and the object API (BENCH r05 object_api).
// run() hands out items [0, n) to the caller and the helpers and returns when every
// item is done.  Helpers spin briefly for the next job (the one-shot's two copy
// phases are ~40 us apart), then sleep.  RS_MI355X_COPY_THREADS = helper count
// (default 7; 0: the caller copies alone).  Measured on MI355X boxes (1024:1024 x
// 1 KiB one-shot encode, two rounds, profiles/r06e/oneshot_threads.txt): 0 helpers
// 136 / 176 us, 1: 169 / 136, 3: 120 / 119, 7: 118 / 111 (object API 90-114 us).
class CopyPool {
  public:
    explicit CopyPool(int helpers) {
        for (int i = 0; i < helpers; ++i) th_.emplace_back([this] { worker(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;
    template <typename F>
    void run(uint64_t n, const F &fn) {
        if (n == 0) return;
        if (th_.empty() || n == 1) {
            for (uint64_t i = 0; i < n; ++i) fn(i);
            return;
        }
        std::lock_guard<std::mutex> one(run_mu_);  // one job at a time per pool
        Job job;
        job.n = n;
        job.call = [](const void *f, uint64_t i) { (*static_cast<const F *>(f))(i); };
        job.fn = &fn;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_.store(&job);
            gen_.fetch_add(1);
        }
        cv_.notify_all();
        drain(job);
        while (job.done.load() < n) __builtin_ia32_pause();
        job_.store(nullptr);
        while (users_.load() != 0) __builtin_ia32_pause();  // no helper still holds &job
    }

  private:
    struct Job {
        uint64_t n = 0;
        void (*call)(const void *, uint64_t) = nullptr;
        const void *fn = nullptr;
        std::atomic<uint64_t> next{0}, done{0};
    };
    static void drain(Job &j) {
        for (uint64_t i; (i = j.next.fetch_add(1)) < j.n;) {
            j.call(j.fn, i);
            j.done.fetch_add(1);
        }
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            while (gen_.load() == seen && !stop_.load()) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100)) {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [&] { return gen_.load() != seen || stop_.load(); });
                    break;
                }
                __builtin_ia32_pause();
            }
            if (stop_.load()) return;
            seen = gen_.load();
            users_.fetch_add(1);
            if (Job *j = job_.load()) drain(*j);
            users_.fetch_sub(1);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_;
    std::atomic<Job *> job_{nullptr};
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> users_{0};
    std::atomic<bool> stop_{false};
};

}  // namespace

// ---------------------------------------------------------------------------
struct rs_context {
    int device = 0;
    uint32_t *d_tw = nullptr;
    uint32_t *d_lut = nullptr;
    uint16_t *d_lwfold = nullptr;       // d_lwfold_base + 1 (segments 4-byte aligned)
    uint16_t *d_lwfold_base = nullptr;
    uint16_t lw0 = 0;
    bool mono = true;             // RS_MI355X_NO_MONO=1 disables the column kernel
    bool split = true;            // RS_MI355X_NO_SPLIT=1 disables the split decode plan (A/B)
    bool mono_all = false;        // RS_MI355X_MONO_ALL=1: unstaged column kernel too (see use_mono)
    uint32_t mono_max_packs = 256;   // column kernel only up to this many packs (RS_MI355X_MONO_MAX_PACKS)
    // 2-element packs (rs_mono.hip Fmt<2>) for staged column-kernel decodes of at
    // most this many 4-element packs (RS_MI355X_E2_MAX_PACKS; 0 = never), and
    // for encodes too when e2_encode (measured: tools/e2_probe.py).
    // Default: half the device's CUs, so the doubled workgroup count (one per
    // 2-element pack) still runs in one wave of workgroups -- at 192 packs on 256
    // CUs the 384 workgroups took two: 1024:1024 x 1536 B decode 26.3 -> 15.8 us
    // with 4-element packs (profiles/r04a/e2_max_packs.txt)
    uint32_t e2_max_packs = 128, e2_default = 128;
    bool e2_encode = true;
    // one-row-per-lane column kernel (rs_lane.hip) for single-chunk 2-element
    // encodes of 2^8 .. 2^lane_max_l rows (RS_MI355X_LANE=0/1; rs_mono_enable + 32:
    // on up to 2^10, + 64: off).  Default 2^9: measured against k_mono (tools/lane_ab.py,
    // profiles/r05c): 256:256 x 1 KiB 4.72 -> 4.35 us, 512:512 5.61 -> 5.50 us, but
    // 1024:1024 8.09 -> 8.70 us (its layers' exchange chain is longer than k_mono's)
    bool lane = true, lane_default = true;
    int lane_max_l = 9, lane_max_l_default = 9;
    // half-split 2^12-row transforms (half_split below; RS_MI355X_HALF=0/1;
    // rs_mono_enable + 128: on, + 256: off).  Off by default: measured slower than
    // the pass kernels at every shape tried (4096:4096 x 1 KiB encode 19.5 -> 25.0 us,
    // 2048:2048 x 1 KiB decode 24.8 -> 33.1 us; profiles/r05e/route_half*.jsonl): each
    // half launch stages a whole 2^11-row twiddle image per workgroup (~3 us of
    // load issue, profiles/r05e/half_stamps.txt) where a pass stages its sets' tables
    bool half = false, half_default = false;
    // quad encode (try_quad below; rs_mono.hip kMonoQuadEnc): single-chunk 2-element
    // encodes of 2^10 rows as the 4-element kernel of 2^9 pair rows (RS_MI355X_QUAD=0/1;
    // rs_mono_enable + 2048: on, + 4096: off)
    bool quad = false, quad_default = false;
    // multi-chunk encodes of 2^2..2^7-row transforms on k_chunks (use_chunks below;
    // RS_MI355X_CHUNKS=0/1; rs_mono_enable + 512: on, + 1024: off)
    bool chunks = true, chunks_default = true;
    bool chunks_forced = false;  // every multi-chunk shape k_chunks supports (+ 512)
    bool chunks_forced_default = false;  // RS_MI355X_CHUNKS=2 at context creation
    uint32_t *d_top = nullptr;    // layer-11 perm tables of the half-split kernels (top_table)
    bool pad_small = true;        // decodes of 16..64 work rows on the 2^7-row column kernel (RS_MI355X_PAD_SMALL)
    int chunk_par = -1;           // RS_MI355X_CHUNK_PARALLEL: -1 by pack count (chunk_parallel), 0 / 1 forced
    uint32_t *d_lut2 = nullptr;   // perm2_by_log: the 2-element form of d_lut
    // the pass kernels' tables as 8-word bases (rs_kernels.hip BasisStager; RS_MI355X_PASS_BASIS=1).
    // Off by default: within +-2.5 % of the 20-word tables on 9 pass shapes, slower on the small
    // ones (4096:4096 x 1 KiB decode 100 % 39.4 -> 40.3 us, 8192:8192 x 64 KiB encode 1028 ->
    // 1003 us; profiles/r05h/passbasis_*.jsonl)
    uint32_t *d_twb = nullptr, *d_lutb = nullptr;  // by skew index / by log factor
    bool pass_basis = false;
    std::mutex img_mu;            // guards d_img, d_img2
    uint32_t *d_img[13] = {};     // column-kernel twiddle images per L (built at context creation)
    uint32_t *d_img2[13] = {};    // the same in the 2-element table format
    uint32_t *d_imgb[13] = {};    // 8-word basis images of the 2-element format (basis_images)
    uint32_t *d_imgb4[8] = {};    // the same for the 4-element format, 2^2..2^7 rows
    std::mutex host_engine_mu;  // guards host_engine_buf (rs_engine_*_host staging)
    DevBuf host_engine_buf;
    std::mutex mu;  // guards ws_by_stream (device-resident API scratch), prof, recs
    // at most RS_MAX_STREAM_WORKSPACES entries.  When a further stream arrives,
    // the least recently used entry's workspace is handed to it: first its
    // `done` event (recorded on its stream at the end of each call that used it,
    // ws_release) is waited for -- the event outlives a destroyed stream, and
    // no other stream or context is stalled -- and its buffers are kept, so no
    // hipFree (which synchronizes the device) runs on the call path
    struct WsEntry {
        std::unique_ptr<Workspace> w;
        uint64_t last_use = 0;
        hipEvent_t done = nullptr;
        bool done_valid = false;  // `done` was recorded after the entry's last call
    };
    std::unordered_map<hipStream_t, WsEntry> ws_by_stream;
    uint64_t ws_clock = 0;
    Workspace &ws(hipStream_t s) {  // caller holds mu, on the context's device
        auto it = ws_by_stream.find(s);
        if (it == ws_by_stream.end()) {
            WsEntry e{std::unique_ptr<Workspace>(new Workspace), 0, nullptr, false};
            if (ws_by_stream.size() >= RS_MAX_STREAM_WORKSPACES) {
                auto lru = ws_by_stream.begin();
                for (auto j = ws_by_stream.begin(); j != ws_by_stream.end(); ++j)
                    if (j->second.last_use < lru->second.last_use) lru = j;
                if (lru->second.done_valid) check(hipEventSynchronize(lru->second.done));
                else check(hipDeviceSynchronize());  // last used before the map filled up (see ws_release)
                e.w = std::move(lru->second.w);
                e.done = lru->second.done;
                ws_by_stream.erase(lru);
            }
            it = ws_by_stream.emplace(s, std::move(e)).first;
        }
        it->second.last_use = ++ws_clock;
        return *it->second.w;
    }
    // the call that used ws(s) has enqueued its work: mark the workspace busy
    // until that completes (caller holds mu).  Only once the map is half full --
    // an event record is one more packet on the caller's stream, and a caller
    // with few streams never evicts
    void ws_release(hipStream_t s) {
        auto it = ws_by_stream.find(s);
        if (it == ws_by_stream.end()) return;
        WsEntry &e = it->second;
        e.done_valid = false;
        if (ws_by_stream.size() < RS_MAX_STREAM_WORKSPACES / 2) return;
        if (!e.done && hipEventCreateWithFlags(&e.done, hipEventDisableTiming) != hipSuccess) {
            e.done = nullptr;
            return;
        }
        e.done_valid = hipEventRecord(e.done, s) == hipSuccess;
    }
    void ws_erase(hipStream_t s) {
        auto it = ws_by_stream.find(s);
        if (it == ws_by_stream.end()) return;
        if (it->second.done) (void)hipEventDestroy(it->second.done);
        ws_by_stream.erase(it);
    }
    ~rs_context() {
        for (auto &kv : ws_by_stream)
            if (kv.second.done) (void)hipEventDestroy(kv.second.done);
    }
    // kernel timing (rs_profile_enable)
    // host-memory pipeline (rs_encode_host / rs_decode_host), built on first use
    struct Pipe {
        static constexpr int kStreams = 3;
        hipStream_t st[kStreams] = {};
        Workspace ws[kStreams];
        DevBuf orig, rec, out;
        ~Pipe() {
            for (hipStream_t s : st)
                if (s) (void)hipStreamDestroy(s);
        }
    };
    Pipe *pipe = nullptr;
    // one-shot rs_encode / rs_decode (lib.rs:251-353): the working space of the last calls
    // (pinned staging, device buffers, workspace, stream), handed to the next call's
    // encoder / decoder as an EncoderWork / DecoderWork would be -- no hipHostMalloc,
    // hipMalloc or hipStreamCreate per call, and no hipHostFree / hipFree, which
    // synchronize the device.  At most kOneShotPool of each, freed with the context.
    static constexpr size_t kOneShotPool = 2;
    std::mutex pool_mu;
    std::vector<rs_encoder_work *> enc_pool;
    std::vector<rs_decoder_work *> dec_pool;
    // one-shot shard copies in on the CopyPool too (RS_MI355X_COPYIN_POOL=0: on the calling
    // thread only; the results always go out on the pool)
    bool copyin_pool = true;
    // the one-shot calls' host copies (CopyPool), started on first use
    std::once_flag copy_once;
    std::unique_ptr<CopyPool> copy_pool;
    CopyPool &copies() {
        std::call_once(copy_once, [this] {
            int helpers = 7;
            if (const char *v = getenv("RS_MI355X_COPY_THREADS")) helpers = std::max(0, std::min(15, atoi(v)));
            copy_pool.reset(new CopyPool(helpers));
        });
        return *copy_pool;
    }
    bool prof = false;
    struct Rec {
        hipEvent_t a, b;
        std::string name;
        uint64_t bytes;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    hipEvent_t take_event() {
        if (pool.empty()) {
            hipEvent_t e;
            check(hipEventCreate(&e));
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
};

namespace {
// The workspace of one API call on stream s (caller holds ctx->mu); released
// (rs_context::ws_release) once the call has enqueued its work.
struct StreamWs {
    rs_context *c;
    hipStream_t s;
    Workspace &w;
    StreamWs(rs_context *c_, hipStream_t s_) : c(c_), s(s_), w(c_->ws(s_)) {}
    ~StreamWs() { c->ws_release(s); }
    StreamWs(const StreamWs &) = delete;
    StreamWs &operator=(const StreamWs &) = delete;
};
// Kernel timing (rs_profile_enable): the context of the current API call.
thread_local rs_context *t_prof_ctx = nullptr;
struct ProfScope {
    explicit ProfScope(rs_context *c) { t_prof_ctx = c && c->prof ? c : nullptr; }
    ~ProfScope() { t_prof_ctx = nullptr; }
};
void prof_begin(hipStream_t s, hipEvent_t *ev) {
    *ev = t_prof_ctx->take_event();
    check(hipEventRecord(*ev, s));
}
void prof_end(hipStream_t s, hipEvent_t ev, const char *name, uint64_t bytes) {
    hipEvent_t b = t_prof_ctx->take_event();
    check(hipEventRecord(b, s));
    t_prof_ctx->recs.push_back({ev, b, name, bytes});
}
}  // namespace

namespace {

// Geometry of a transform: `packs` packs of 4 elements each (8 bytes: 4 low +
// 4 high) per row; work buffers use rows of `stride` bytes.  The caller's
// matrices may be column slices of wider ones: their own row strides (0 =
// `stride`).
struct Geom {
    uint64_t stride;
    uint32_t packs;
    uint64_t orig_stride = 0, rec_stride = 0, out_stride = 0;
    // a batch of stripes of this shape: stripe b's matrices start b * *_bstride
    // bytes after the base pointers (rs_encode_device_batch / rs_decode_device_batch)
    uint32_t stripes = 1;
    uint64_t orig_bstride = 0, rec_bstride = 0, out_bstride = 0;
    rs::ShardFormat fmt;  // byte layout of the caller's matrices (tails, alignment)
    uint64_t orig() const { return orig_stride ? orig_stride : stride; }
    uint64_t rec() const { return rec_stride ? rec_stride : stride; }
    uint64_t out() const { return out_stride ? out_stride : stride; }
};

// Packs of a shard of S bytes: 8 per whole 64-byte block, then one per 4
// elements of the tail block (S % 64 bytes = (S % 64) / 2 elements).
uint32_t packs_of(uint64_t S) { return uint32_t(S / 64 * 8 + ((S % 64) / 2 + 3) / 4); }

// Geometry of a device call on the caller's matrices of shards of S bytes
// (any even S: the tail block follows the reference's layout,
// src/engine/shards.rs:38-74; rs_device.hpp ShardFormat).  Strides 0 = S.
// Work buffers use rows of whole 64-byte blocks.
Geom device_geom(uint64_t S, uint64_t orig_stride, uint64_t rec_stride, uint64_t out_stride,
                 std::initializer_list<const void *> ptrs) {
    Geom g{round_up(S, 64), packs_of(S)};
    g.orig_stride = orig_stride ? orig_stride : S;
    g.rec_stride = rec_stride ? rec_stride : S;
    g.out_stride = out_stride ? out_stride : S;
    bool aligned = g.orig_stride % 4 == 0 && g.rec_stride % 4 == 0 && g.out_stride % 4 == 0;
    for (const void *p : ptrs) aligned = aligned && (reinterpret_cast<uintptr_t>(p) & 3) == 0;
    if (S % 64 || !aligned) {
        g.fmt.full_packs = uint32_t(S / 64 * 8);
        g.fmt.tail_h = uint32_t(S % 64 / 2);
        g.fmt.io_bytes = aligned ? 0 : 1;
    }
    return g;
}

rs::PassArgs base_args(rs_context *ctx, const Geom &g, uint32_t n) {
    rs::PassArgs A;
    A.n = n;
    A.packs = g.packs;
    A.slices = (g.packs + 63) / 64;
    A.tw = ctx->pass_basis ? ctx->d_twb : ctx->d_tw;
    A.lut = ctx->pass_basis ? ctx->d_lutb : ctx->d_lut;
    A.tab_basis = ctx->pass_basis ? 1u : 0u;
    A.fmt = g.fmt;
    return A;
}

// Split of a 2^L-row transform into bit levels of at most kMaxK bits each,
// low to high: level k covers transform-row bits [lo_k, lo_k + K_k).  The
// IFFT runs levels 0..m-1 ascending, the FFT m-1..0 descending; the top
// level's IFFT + FFT are fused into one pass (DESIGN.md "Pass structure").
constexpr uint32_t kMaxK = 8;  // pass kernels exist for K <= 8
constexpr uint64_t kMaxBatchStripes = 65535;  // stripes per column-kernel launch (grid.y)
uint32_t g_max_k = 0;  // RS_MI355X_MAX_K (4..8) overrides the choice below
// Measured with the pruned decode passes (profiles/r01p/ab_maxk_*, tools/ab_maxk.sh):
// encodes run fastest with 8-bit levels (32768:32768 x 1 KiB 671 -> 711 GiB/s vs 7),
// decodes with 6-bit levels (8192:8192 x 64 KiB 1 % / 100 %: 637 / 531 -> 840 / 641 GiB/s:
// more levels below the top, so more of the FFT is pruned and more IFFT blocks skipped)
uint32_t max_k_enc(uint32_t) { return g_max_k ? g_max_k : 8; }
// 2^13 work rows of short shards take two 7 + 6-bit levels instead of three
// (5 + 4 + 4): two fewer launches.  4096:4096 x 1 KiB decode 46.1 / 43.2 ->
// 40.4 / 38.5 us at 1 % / 100 % loss; at 2^14 and up 7-bit levels lost (8192:8192
// x 1 KiB 70.3 -> 72.7 us, 1000:10000 49.5 -> 62.0 us; profiles/r04a/ab_maxk_shapes.txt)
uint32_t max_k_dec(uint32_t u = 0, uint32_t packs = 0) {
    if (g_max_k) return g_max_k;
    return u == 13 && packs <= 512 ? 7 : 6;
}
struct Levels {
    uint32_t m = 0;
    uint32_t lo[4] = {0, 0, 0, 0}, K[4] = {0, 0, 0, 0};
};
Levels levels(uint32_t L, uint32_t mk) {
    Levels v;
    v.m = L == 0 ? 1 : (L + mk - 1) / mk;
    // the fused top level does two transforms: give it the smallest share
    uint32_t rest = L;
    for (uint32_t k = 0; k < v.m; ++k) {
        const uint32_t left = v.m - k;
        v.K[k] = (rest + left - 1) / left;
        v.lo[k] = L - rest;
        rest -= v.K[k];
    }
    return v;
}

// Algorithmic HBM bytes of one pass: rows it must read + rows it writes.
uint64_t pass_bytes(int K, const rs::PassArgs &A, uint64_t decode_rows_read, uint64_t decode_rows_written) {
    const uint64_t span = uint64_t(A.n) * (A.grid_chunks + A.in_chunks + A.out_chunks - 2);
    uint64_t rd = 0, wr = 0;
    if (A.work_in) rd = (uint64_t(A.nsets) << K) * A.grid_chunks * A.in_chunks;
    else if (decode_rows_read) rd = decode_rows_read;
    else
        for (uint32_t k = 0; k < A.nsrc; ++k)
            rd += std::min<uint64_t>(A.src[k].row_end, span) - std::min<uint64_t>(A.src[k].row_begin, span);
    if (A.xor_in) rd += uint64_t(A.nsets) << K;
    if (A.work_out) wr = (uint64_t(A.nsets) << K) * A.grid_chunks * A.out_chunks;
    else if (decode_rows_written) wr = decode_rows_written;
    else wr = std::min<uint64_t>(A.dst.row_end, span) - std::min<uint64_t>(A.dst.row_begin, span);
    const uint64_t row = uint64_t(A.packs) * 8;
    return (rd + wr) * row;
}

void launch(int K, int flags, rs::PassArgs A, uint32_t nsets, uint32_t a, hipStream_t s, uint64_t dec_rd = 0,
            uint64_t dec_wr = 0) {
    A.nsets = nsets;
    A.a = a;
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_pass(K, flags, A, s));
    if (t_prof_ctx) prof_end(s, ev, rs::launch_name_buf(), pass_bytes(K, A, dec_rd, dec_wr));
}

// One pass over bit level k of a 2^L-row transform (n rows per chunk).
void run_level(rs::PassArgs A, const Levels &lv, uint32_t k, int flags, uint32_t n, hipStream_t s,
               uint64_t dec_rd = 0, uint64_t dec_wr = 0) {
    launch(lv.K[k], flags, A, n >> lv.K[k], lv.lo[k], s, dec_rd, dec_wr);
}

// Column kernel (rs_mono.hip): twiddle images of a 2^L-row transform for
// every skew offset t * n, t = 0 .. 65536/n - 1 (rs_device.hpp), built on the
// host from the skew tables once per context and L.
constexpr uint32_t kMonoMinL = 7, kMonoMaxL = 12;
constexpr uint32_t kChunksMinL = 2;  // k_chunks' smallest transform (images built from here)
constexpr uint32_t kChunksMaxWaves = 8;  // k_chunks' waves per workgroup (rs_chunks.hip kMaxWaves)
const uint32_t *mono_images(rs_context *ctx, uint32_t L, uint32_t elems = 4) {
    std::lock_guard<std::mutex> lock(ctx->img_mu);
    uint32_t *&slot_ptr = elems == 2 ? ctx->d_img2[L] : ctx->d_img[L];
    if (slot_ptr) return slot_ptr;
    const rs::GfTables &T = rs::tables();
    const std::vector<uint32_t> &src = elems == 2 ? T.perm2_by_skew : T.perm_by_skew;
    const size_t tw = elems == 2 ? rs::kPerm2Words : rs::kPermWords;
    const uint32_t n = 1u << L, nimg = 65536u / n;  // skew offsets t * n + (n - 2) <= 65534
    const size_t words = size_t(n - 1) * tw;
    std::vector<uint32_t> h(words * nimg);
    for (uint32_t t = 0; t < nimg; ++t) {
        uint32_t *dst = &h[t * words];
        for (uint32_t b = 0; b < L; ++b)
            for (uint32_t g = 0; g < (n >> (b + 1)); ++g) {
                const uint32_t slot = n - (n >> b) + g;
                const uint32_t idx = (g << (b + 1)) + (1u << b) + t * n - 1;
                std::copy_n(&src[size_t(idx) * tw], tw, dst + size_t(slot) * tw);
            }
    }
    uint32_t *d = nullptr;
    check(hipMalloc(&d, h.size() * 4));
    check(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    slot_ptr = d;
    return d;
}

// Basis images (the 2-element staged kernels' twiddles: k_mono, rs_mono.hip
// basis_expand, and k_chunks): the layout of mono_images, 8 words per table -- the
// products P(e_i) = x * e_i of the table's multiplier with the 16 Cantor basis
// elements, word 2f = P(e_2f) | P(e_2f+1) << 16 (the low byte's 2-bit field f),
// word 2f + 1 = P(e_8+2f) | P(e_9+2f) << 16 (the high byte's); zero for skew 65535.
// 4-element format (rs_chunks.hip CTabsBasis4): per input byte B, words 4B .. 4B + 3 =
// P0 | P1 << 16, P3 | P4 << 16, P6 | P7 << 16, P2 | P5 << 16 with Pj = P(e_8B+j).
constexpr uint32_t kBasisWords = 8;
// The 4-element basis of multiplier log lm (rs_gf.hpp basis4_expand's layout); zero
// when !nonzero or lm = 65535 as a skew (multiply by zero)
void basis4_words(const rs::GfTables &T, uint32_t lm, bool nonzero, uint32_t *o) {
    auto P = [&](int i) -> uint32_t {
        return !nonzero || lm > 65535u ? 0u : T.mul(uint16_t(1u << i), uint16_t(lm));
    };
    for (int B = 0; B < 2; ++B) {
        const int j = 8 * B;
        o[4 * B] = P(j) | (P(j + 1) << 16);
        o[4 * B + 1] = P(j + 3) | (P(j + 4) << 16);
        o[4 * B + 2] = P(j + 6) | (P(j + 7) << 16);
        o[4 * B + 3] = P(j + 2) | (P(j + 5) << 16);
    }
}
// The pass kernels' basis tables (PassArgs::tab_basis): 4-element bases by skew
// index (zero for skew 65535) and by log factor; built when first needed.
void pass_basis_tables(rs_context *ctx) {
    std::lock_guard<std::mutex> lock(ctx->img_mu);
    if (ctx->d_twb) return;
    const rs::GfTables &T = rs::tables();
    std::vector<uint32_t> tw(size_t(65536) * kBasisWords), lu(size_t(65536) * kBasisWords);
    for (uint32_t i = 0; i < 65536; ++i) {
        basis4_words(T, i < 65535 ? T.skew[i] : 65535u, i < 65535 && T.skew[i] != 65535, &tw[size_t(i) * kBasisWords]);
        basis4_words(T, uint16_t(i), true, &lu[size_t(i) * kBasisWords]);
    }
    check(hipMalloc(&ctx->d_lutb, lu.size() * 4));
    check(hipMemcpy(ctx->d_lutb, lu.data(), lu.size() * 4, hipMemcpyHostToDevice));
    uint32_t *d = nullptr;
    check(hipMalloc(&d, tw.size() * 4));
    check(hipMemcpy(d, tw.data(), tw.size() * 4, hipMemcpyHostToDevice));
    ctx->d_twb = d;
}
const uint32_t *basis_images(rs_context *ctx, uint32_t L, uint32_t elems = 2) {
    std::lock_guard<std::mutex> lock(ctx->img_mu);
    uint32_t *&slot_ptr = elems == 2 ? ctx->d_imgb[L] : ctx->d_imgb4[L];
    if (slot_ptr) return slot_ptr;
    const rs::GfTables &T = rs::tables();
    const uint32_t n = 1u << L, nimg = 65536u / n;
    const size_t words = size_t(n - 1) * kBasisWords;
    std::vector<uint32_t> h(words * nimg);
    for (uint32_t t = 0; t < nimg; ++t) {
        uint32_t *dst = &h[t * words];
        for (uint32_t b = 0; b < L; ++b)
            for (uint32_t g = 0; g < (n >> (b + 1)); ++g) {
                const uint32_t slot = n - (n >> b) + g;
                const uint32_t idx = (g << (b + 1)) + (1u << b) + t * n - 1;
                const uint16_t lm = T.skew[idx];
                auto P = [&](int i) -> uint32_t { return lm == 65535 ? 0u : T.mul(uint16_t(1u << i), lm); };
                uint32_t *o = dst + size_t(slot) * kBasisWords;
                if (elems == 2) {
                    for (uint32_t f = 0; f < 4; ++f) {
                        o[2 * f] = P(int(2 * f)) | (P(int(2 * f + 1)) << 16);
                        o[2 * f + 1] = P(int(8 + 2 * f)) | (P(int(9 + 2 * f)) << 16);
                    }
                } else {
                    for (int B = 0; B < 2; ++B) {
                        const int j = 8 * B;
                        o[4 * B] = P(j) | (P(j + 1) << 16);
                        o[4 * B + 1] = P(j + 3) | (P(j + 4) << 16);
                        o[4 * B + 2] = P(j + 6) | (P(j + 7) << 16);
                        o[4 * B + 3] = P(j + 2) | (P(j + 5) << 16);
                    }
                }
            }
    }
    uint32_t *d = nullptr;
    check(hipMalloc(&d, h.size() * 4));
    check(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    slot_ptr = d;
    return d;
}

// The column kernel runs where it beats the pass kernels: its staged
// variant (one chunk, L <= 10).  RS_MI355X_MONO_ALL=1 also routes multi-chunk
// and L = 11, 12 transforms to its unstaged variant (tests, tuning).
bool use_mono(rs_context *ctx, uint32_t L, const Geom &g, uint32_t chunks) {
    if (!ctx->mono || L < kMonoMinL || L > kMonoMaxL || g.packs > ctx->mono_max_packs) return false;
    return ctx->mono_all || rs::mono_staged(int(L), chunks);
}

// Staged transforms of few packs use 2-element packs: twice the workgroups on
// a chip whose CUs the 4-element packs leave idle (rs_mono.hip Fmt).  Decodes
// since round 2 (14.6 vs 15.4 us, now 13.8); encodes since round 4, when they
// measured faster too (1024:1024 x 1 KiB 8.11 -> 7.96 us, 512:512 6.1 -> 5.7,
// 1024:1024 x 256 B 8.0 -> 7.3; profiles/r04a/e2_encode_ab.txt) -- in rounds 2
// and 3 the encode was slower (9.4 vs 8.4 us), then about equal (8.5-8.8 vs
// 8.4-8.75 us).
rs::MonoArgs mono_args(rs_context *ctx, uint32_t L, const Geom &g, bool staged, bool decode = false) {
    rs::MonoArgs M;
    // (a batch's stripes already fill the chip: the bound covers all its packs)
    const bool e2 = staged && (decode || ctx->e2_encode) && uint64_t(g.packs) * g.stripes <= ctx->e2_max_packs &&
                    L <= 11;
    M.elems = e2 ? 2 : 4;
    // 2-element packs: two per 4-element pack of the whole blocks, one per 2 tail elements
    M.packs = !e2 ? g.packs
                  : g.fmt.full_packs == 0xFFFFFFFFu ? 2 * g.packs : 2 * g.fmt.full_packs + (g.fmt.tail_h + 1) / 2;
    M.packs_per_xcd = (M.packs + 7) / 8;
    M.stripes = g.stripes;  // a batch of stripes runs in one launch
    // 2-element packs with RS_MONO_BASIS: basis images (rs_mono.hip Stage::kBasis builds the tables)
    const bool basis = e2 && RS_MONO_BASIS;
    M.img = basis ? basis_images(ctx, L) : mono_images(ctx, L, M.elems);
    M.img_words = uint64_t((1u << L) - 1) * (basis ? kBasisWords : e2 ? rs::kPerm2Words : rs::kPermWords);
    M.lut = e2 ? ctx->d_lut2 : ctx->d_lut;
    M.fmt = g.fmt;
    return M;
}

void launch_mono(int mode, uint32_t L, const rs::MonoArgs &M, hipStream_t s, uint64_t bytes) {
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_mono(mode, int(L), M, s));
    if (t_prof_ctx) prof_end(s, ev, rs::launch_name_buf(), bytes);
}

// A single-chunk encode goes to the lane kernel (rs_lane.hip) when enabled and
// its column arguments are 2-element packs of 2^8..2^10 rows; false: not taken.
bool try_lane(rs_context *ctx, uint32_t L, uint32_t chunks, const rs::MonoArgs &M, hipStream_t s, uint64_t bytes) {
    if (!ctx->lane || chunks != 1 || M.elems != 2 || int(L) > ctx->lane_max_l || !rs::lane_supported(int(L)))
        return false;
    rs::MonoArgs F = M;  // the lane kernel stages basis or 16-word images (RS_LANE_BASIS)
    F.img = RS_LANE_BASIS ? basis_images(ctx, L, 2) : mono_images(ctx, L, 2);
    F.img_words = uint64_t((1u << L) - 1) * (RS_LANE_BASIS ? kBasisWords : rs::kPerm2Words);
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_lane(int(L), F, s));
    if (t_prof_ctx) prof_end(s, ev, rs::launch_name_buf(), bytes);
    return true;
}

// A single-chunk 2-element encode of 2^10 rows goes to the quad form of the column
// kernel (rs_mono.hip kMonoQuadEnc: the 4-element kernel of 2^9 pair rows, each
// pack 2 elements x 2 rows) when enabled; false: not taken.  Its images: the
// 4-element tables of layers >= 1 (the 2^L-row image from slot 2^(L-1) on) and
// the 2-element layer-0 tables (A.lut).
bool try_quad(rs_context *ctx, uint32_t L, uint32_t chunks, const rs::MonoArgs &M, hipStream_t s, uint64_t bytes) {
    if (!ctx->quad || chunks != 1 || M.elems != 2 || !rs::quad_supported(int(L))) return false;
    rs::MonoArgs Q = M;
    const uint64_t n = uint64_t(1) << L;
    Q.img = mono_images(ctx, L, 4) + (n / 2) * rs::kPermWords;
    Q.img_words = (n - 1) * rs::kPermWords;
    Q.lut = mono_images(ctx, L, 2);
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_quad(int(L), Q, s));
    if (t_prof_ctx) prof_end(s, ev, rs::launch_name_buf(), bytes);
    return true;
}

// Multi-chunk encodes of small transforms (rs_chunks.hip): one launch in which the
// waves of a pack's workgroup take the chunks in parallel (HighRate input chunks,
// LowRate output chunks), twiddle tables built in LDS from basis images.  One
// stripe; the column kernel's pack bound.  Measured against the passes (wall us
// per call, profiles/r05h/chunks{,4}_{forced,none}.jsonl): 1000:100 x 1 KiB 13.2 ->
// 6.5, x 2 KiB 13.5 -> 7.8; 9000:100 x 1 / 2 KiB 35.2 / 57.0 -> 21.1 / 24.7; 100:10
// 7.9 -> 4.9; LowRate 128:1024 x 1 / 2 KiB 8.2 / 8.6 -> 6.2 / 7.3.  The exception,
// LowRate with 2-element packs past 8 output chunks (64:640 5.86 / 5.87, 100:9000
// x 1 KiB 21.7 -> 22.6), stays on the pass.  rs_mono_enable + 512 / RS_MI355X_CHUNKS=2:
// every supported shape.
bool use_chunks(rs_context *ctx, uint32_t L, const Geom &g, uint32_t chunks, bool high) {
    // (RS_MI355X_CHUNK_PARALLEL forces one of the pass forms: tests, A/B)
    // (HighRate up to twice the pack bound, two packs per wave: 1000:100 x 4 KiB 13.7 -> 9.3 us,
    // profiles/r05h/chunks4_pw.txt; LowRate there lost, 8.8 -> 10.2)
    if (!ctx->chunks || !ctx->mono || ctx->mono_all || ctx->chunk_par >= 0 || chunks < 2 || g.stripes != 1 ||
        !rs::chunks_supported(int(L)) || g.packs > (high ? 2 : 1) * ctx->mono_max_packs)
        return false;
    const bool e2 = ctx->e2_encode && uint64_t(g.packs) <= ctx->e2_max_packs;  // as mono_args decides
    return ctx->chunks_forced || high || !e2 || chunks <= kChunksMaxWaves;
}
void launch_chunks(rs_context *ctx, const Geom &g, bool high, uint32_t L, const rs::RowMap &src, const rs::RowMap &dst,
                   uint32_t chunks, uint64_t bytes, hipStream_t s) {
    rs::MonoArgs Mo = mono_args(ctx, L, g, true);
    // basis images, expanded in the kernel (rs_chunks.hip CTabsBasis / CTabsBasis4)
    Mo.img = basis_images(ctx, L, Mo.elems);
    Mo.img_words = uint64_t((1u << L) - 1) * kBasisWords;
    Mo.src[0] = src;
    Mo.nsrc = 1;
    Mo.dst = dst;
    Mo.chunks = chunks;
    Mo.ifft_img = high ? 1 : 0;  // HighRate chunk c: skew offset c n + n; LowRate: 0
    Mo.ifft_img_step = high ? 1 : 0;
    Mo.fft_img = high ? 0 : 1;  // LowRate output chunk c: skew offset c n + n
    Mo.fft_img_step = high ? 0 : 1;
    const int pw = g.packs > ctx->mono_max_packs ? 2 : 1;  // packs per wave (use_chunks' wide shapes)
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_chunks(int(L), high, Mo, s, pw));
    if (t_prof_ctx) prof_end(s, ev, rs::launch_name_buf(), bytes);
}

// Half-split transforms of 2^12 rows (rs_mono.hip kMonoHalf*):
// the 2^11-row column kernel twice -- kMonoHalfI* runs the IFFT's layers 0..10
// of each half that holds input rows into the work rows, kMonoHalfF* the top
// layer (IFFT layer 11, the decode's formal derivative, FFT layer 11) and the
// FFT's layers 10..0 of each half that holds output rows.  Two launches instead
// of the pass kernels' three (two for the levels below the top + the fused top)
// and no separate eval_poly-free row pass; the work rows are written and read
// once.  Single chunk, one stripe.
constexpr uint32_t kTopTables = 31;  // skew indices 2047 + 2048 j <= 63487 (65535 entries)
bool use_half(rs_context *ctx, uint32_t L, const Geom &g, uint32_t chunks) {
    // (rs_mono_enable 2, MONO_ALL: the unstaged 2^12-row column kernel instead)
    return ctx->half && ctx->mono && !ctx->mono_all && L == 12 && chunks == 1 && g.stripes == 1 && g.packs <= ctx->mono_max_packs &&
           rs::mono_staged(11, 1);
}
// The top layer's perm table of a transform with skew offset delta (a multiple
// of 2048): skew index delta + 2047 (engine_naive.rs ifft / fft at dist 2^11).
const uint32_t *top_table(rs_context *ctx, uint32_t delta, uint32_t elems) {
    const uint32_t j = delta / 2048;
    return elems == 2 ? ctx->d_top + kTopTables * rs::kPermWords + j * rs::kPerm2Words : ctx->d_top + j * rs::kPermWords;
}
void launch_half(int mode, uint32_t halves, const rs::MonoArgs &M, hipStream_t s, uint64_t bytes) {
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_mono_half(mode, halves, M, s));
    if (t_prof_ctx) prof_end(s, ev, rs::launch_name_buf(), bytes);
}
// in_halves / out_halves: bit h = half h holds input rows (received rows) /
// output rows (recovery rows, erased originals); i_delta / f_delta: the IFFT's /
// FFT's skew offset; rowinfo (decodes): eval_poly's output for the 4096 rows.
void half_split(rs_context *ctx, Workspace &ws, const Geom &g, bool dec, uint32_t i_delta, uint32_t f_delta,
                const rs::RowMap *src, uint32_t nsrc, const rs::RowMap &dst, const uint32_t *rowinfo,
                uint32_t in_halves, uint32_t out_halves, uint64_t in_rows, uint64_t out_rows, hipStream_t s) {
    if (!in_halves || !out_halves) return;
    uint8_t *W = static_cast<uint8_t *>(ws.buf[0].get(size_t(4096) * g.stride));
    Geom g2 = g;
    g2.stripes = 2;  // the 2-element decision counts both halves' workgroups
    rs::MonoArgs M = mono_args(ctx, 11, g2, true, dec);
    M.stripes = 1;
    M.rowinfo = rowinfo;
    M.top_i = top_table(ctx, i_delta, M.elems);
    M.top_f = top_table(ctx, f_delta, M.elems);
    M.zero_halves = 3u & ~in_halves;
    const uint64_t row = uint64_t(g.packs) * 8;
    const uint32_t nin = uint32_t(__builtin_popcount(in_halves)), nout = uint32_t(__builtin_popcount(out_halves));
    rs::MonoArgs I = M;
    for (uint32_t k = 0; k < nsrc; ++k) I.src[k] = src[k];
    I.nsrc = nsrc;
    I.dst = rs::RowMap{W, g.stride, 0, 4096};
    I.ifft_img = i_delta / 2048;
    I.ifft_img_step = 1;
    I.half0 = in_halves == 2 ? 1 : 0;
    launch_half(dec ? rs::kMonoHalfIDec : rs::kMonoHalfIEnc, nin, I, s, (in_rows + 2048 * nin) * row);
    rs::MonoArgs F = M;
    F.src[0] = rs::RowMap{W, g.stride, 0, 4096};
    F.nsrc = 1;
    F.dst = dst;
    F.fft_img = f_delta / 2048;
    F.fft_img_step = 1;
    F.out_half = out_halves == 2 ? 1 : 0;
    launch_half(dec ? rs::kMonoHalfFDec : rs::kMonoHalfFEnc, nout, F, s, (2048 * nin + out_rows) * row);
}
// halves of [b, e) in a 4096-row transform
uint32_t halves_of(uint64_t b, uint64_t e) { return b >= e ? 0u : (b < 2048 ? 1u : 0u) | (e > 2048 ? 2u : 0u); }

// Single-level multi-chunk encodes: spread the chunks over the grid (grid.y)
// when the packs alone give few workgroups (RS_MI355X_CHUNK_PARALLEL = 0 / 1
// forces the serial / parallel form; tools/ab_chunks.sh measures the threshold).
// The HighRate parallel form needs a work buffer of every chunk's IFFT rows
// (`scratch` bytes, about the size of the input); past kChunkParallelMaxScratch
// the serial form runs instead, which needs none (60000:100 x 32 KiB would
// otherwise allocate ~1.9 GB per stream).
constexpr uint32_t kChunkParallelMaxPacks = 4096;
constexpr uint64_t kChunkParallelMaxScratch = uint64_t(256) << 20;
bool chunk_parallel(rs_context *ctx, const Geom &g, uint64_t scratch = 0) {
    if (ctx->chunk_par >= 0) return ctx->chunk_par != 0;
    return g.packs <= kChunkParallelMaxPacks && scratch <= kChunkParallelMaxScratch;
}

// HighRate encode (rate_high.rs:44-87) from device rows to device rows:
// chunk c's IFFT uses skew_delta c*n + n, the chunks are XOR-folded, one FFT
// with skew_delta 0 produces the recovery rows.
void encode_high(rs_context *ctx, Workspace &ws, const Geom &g, uint64_t N, uint64_t M, const uint8_t *orig,
                 uint8_t *rec, hipStream_t s) {
    const uint32_t n = uint32_t(next_pow2(M)), L = ilog2(n);
    const uint32_t C = uint32_t((N + n - 1) / n);
    if (g.stripes > 1 && !(use_mono(ctx, L, g, C) && rs::mono_staged(int(L), C))) {  // batch: one stripe after another
        Geom g1 = g;
        g1.stripes = 1;
        for (uint32_t b = 0; b < g.stripes; ++b)
            encode_high(ctx, ws, g1, N, M, orig + b * g.orig_bstride, rec + b * g.rec_bstride, s);
        return;
    }
    const Levels lv = levels(L, max_k_enc(g.packs));
    rs::PassArgs A = base_args(ctx, g, n);
    A.ifft_delta = n;
    A.ifft_delta_step = n;
    const rs::RowMap src{orig, g.orig(), 0, uint32_t(N)}, dst{rec, g.rec(), 0, uint32_t(M)};
    if (use_mono(ctx, L, g, C)) {
        rs::MonoArgs Mo = mono_args(ctx, L, g, rs::mono_staged(int(L), C));
        Mo.src[0] = src;
        Mo.src_bstride[0] = g.orig_bstride;
        Mo.nsrc = 1;
        Mo.dst = dst;
        Mo.dst_bstride = g.rec_bstride;
        Mo.chunks = C;
        Mo.ifft_img = 1;  // chunk c: skew offset c * n + n
        Mo.ifft_img_step = 1;
        Mo.fft_img = 0;
        const uint64_t bytes = (N + M) * uint64_t(g.packs) * 8 * g.stripes;
        if (!try_quad(ctx, L, C, Mo, s, bytes) && !try_lane(ctx, L, C, Mo, s, bytes))
            launch_mono(rs::kMonoEncodeHigh, L, Mo, s, bytes);
        return;
    }
    if (use_chunks(ctx, L, g, C, true)) {
        launch_chunks(ctx, g, true, L, src, dst, C, (N + M) * uint64_t(g.packs) * 8, s);
        return;
    }
    if (use_half(ctx, L, g, C)) {  // IFFT skew n, FFT skew 0
        half_split(ctx, ws, g, false, n, 0, &src, 1, dst, nullptr, halves_of(0, N), halves_of(0, M), N, M, s);
        return;
    }
    if (lv.m == 1 && (C == 1 || !chunk_parallel(ctx, g, uint64_t(C) * n * g.stride))) {
        A.src[0] = src;
        A.nsrc = 1;
        A.in_chunks = C;
        A.dst = dst;
        run_level(A, lv, 0, rs::kIfft | rs::kFft, n, s);
        return;
    }
    uint8_t *W = static_cast<uint8_t *>(ws.buf[0].get(size_t(C) * n * g.stride));
    if (lv.m == 1) {
        // one level, several chunks, few packs: every chunk's IFFT in its own
        // workgroups (grid.y = chunk) into the work rows, then one pass XOR-folds
        // the chunks and runs the FFT -- instead of one workgroup transforming
        // the chunks one after another
        A.work_stride = g.stride;
        rs::PassArgs P = A;
        P.grid_chunks = C;
        P.src[0] = src;
        P.nsrc = 1;
        P.work_out = W;
        run_level(P, lv, 0, rs::kIfft, n, s);
        rs::PassArgs T = A;
        T.work_in = W;
        T.in_chunks = C;
        T.dst = dst;
        run_level(T, lv, 0, rs::kFft, n, s);
        return;
    }
    A.work_stride = g.stride;
    for (uint32_t k = 0; k + 1 < lv.m; ++k) {  // IFFT, low levels, every chunk
        rs::PassArgs P = A;
        P.grid_chunks = C;
        if (k == 0) P.src[0] = src, P.nsrc = 1;
        else P.work_in = W;
        P.work_out = W;
        run_level(P, lv, k, rs::kIfft, n, s);
    }
    rs::PassArgs T = A;  // top level: IFFT per chunk, XOR-fold, FFT
    T.work_in = W;
    T.in_chunks = C;
    T.work_out = W;
    run_level(T, lv, lv.m - 1, rs::kIfft | rs::kFft, n, s);
    for (int k = int(lv.m) - 2; k >= 0; --k) {  // FFT, low levels
        rs::PassArgs P = A;
        P.work_in = W;
        if (k == 0) P.dst = dst;
        else P.work_out = W;
        run_level(P, lv, k, rs::kFft, n, s);
    }
}

// LowRate encode (rate_low.rs:44-87): one IFFT (skew 0), then output chunk c
// is FFT'd with skew_delta c*n + n.
void encode_low(rs_context *ctx, Workspace &ws, const Geom &g, uint64_t N, uint64_t M, const uint8_t *orig,
                uint8_t *rec, hipStream_t s) {
    const uint32_t n = uint32_t(next_pow2(N)), L = ilog2(n);
    const uint32_t C = uint32_t((M + n - 1) / n);
    if (g.stripes > 1 && !(use_mono(ctx, L, g, C) && rs::mono_staged(int(L), C))) {  // batch: one stripe after another
        Geom g1 = g;
        g1.stripes = 1;
        for (uint32_t b = 0; b < g.stripes; ++b)
            encode_low(ctx, ws, g1, N, M, orig + b * g.orig_bstride, rec + b * g.rec_bstride, s);
        return;
    }
    const Levels lv = levels(L, max_k_enc(g.packs));
    rs::PassArgs A = base_args(ctx, g, n);
    A.fft_delta = n;
    A.fft_delta_step = n;
    const rs::RowMap src{orig, g.orig(), 0, uint32_t(N)}, dst{rec, g.rec(), 0, uint32_t(M)};
    if (use_mono(ctx, L, g, C)) {
        rs::MonoArgs Mo = mono_args(ctx, L, g, rs::mono_staged(int(L), C));
        Mo.src[0] = src;
        Mo.src_bstride[0] = g.orig_bstride;
        Mo.nsrc = 1;
        Mo.dst = dst;
        Mo.dst_bstride = g.rec_bstride;
        Mo.chunks = C;
        Mo.ifft_img = 0;
        Mo.fft_img = 1;  // output chunk c: skew offset c * n + n
        Mo.fft_img_step = 1;
        const uint64_t bytes = (N + M) * uint64_t(g.packs) * 8 * g.stripes;
        if (!try_quad(ctx, L, C, Mo, s, bytes) && !try_lane(ctx, L, C, Mo, s, bytes))
            launch_mono(rs::kMonoEncodeLow, L, Mo, s, bytes);
        return;
    }
    if (use_chunks(ctx, L, g, C, false)) {
        launch_chunks(ctx, g, false, L, src, dst, C, (N + M) * uint64_t(g.packs) * 8, s);
        return;
    }
    if (use_half(ctx, L, g, C)) {  // IFFT skew 0, FFT skew n
        half_split(ctx, ws, g, false, 0, n, &src, 1, dst, nullptr, halves_of(0, N), halves_of(0, M), N, M, s);
        return;
    }
    if (lv.m == 1) {
        A.src[0] = src;
        A.nsrc = 1;
        A.dst = dst;
        if (C > 1 && chunk_parallel(ctx, g)) {
            // one level, several output chunks, few packs: each output chunk's
            // workgroups (grid.y) run the IFFT of the originals themselves and that
            // chunk's FFT -- instead of one workgroup running the chunks' FFTs one
            // after another
            A.grid_chunks = C;
            A.in_chunk0 = 1;
        } else {
            A.out_chunks = C;
        }
        run_level(A, lv, 0, rs::kIfft | rs::kFft, n, s);
        return;
    }
    uint8_t *W = static_cast<uint8_t *>(ws.buf[0].get(size_t(n) * g.stride));
    uint8_t *W2 = static_cast<uint8_t *>(ws.buf[1].get(size_t(C) * n * g.stride));
    A.work_stride = g.stride;
    for (uint32_t k = 0; k + 1 < lv.m; ++k) {
        rs::PassArgs P = A;
        if (k == 0) P.src[0] = src, P.nsrc = 1;
        else P.work_in = W;
        P.work_out = W;
        run_level(P, lv, k, rs::kIfft, n, s);
    }
    rs::PassArgs T = A;  // top level: IFFT, then FFT once per output chunk
    T.work_in = W;
    T.out_chunks = C;
    T.work_out = W2;
    run_level(T, lv, lv.m - 1, rs::kIfft | rs::kFft, n, s);
    for (int k = int(lv.m) - 2; k >= 0; --k) {
        rs::PassArgs P = A;
        P.grid_chunks = C;
        P.work_in = W2;
        if (k == 0) P.dst = dst;
        else P.work_out = W2;
        run_level(P, lv, k, rs::kFft, n, s);
    }
}

// FFT passes of a multi-level decode, pruned to the rows that reach an output.
// The last pass stores only erased originals; the pass at level k (bits
// [lo_k, lo_k + K_k)) feeds the lower levels only within aligned superblocks
// of 2^(lo_k + K_k) rows, and its row sets {s_lo + j 2^lo_k + s_hi 2^(lo_k+K_k)}
// (set = s_lo + s_hi 2^lo_k) lie in superblock s_hi.  A superblock holding no
// erased row in the restored range is not launched; the needed ones go out as
// at most kFftRuns launches of consecutive sets (smallest gaps bridged first).
// A pruned FFT: the reference transforms every row (rate_high.rs:241-246) and
// reads back only the erased ones, so the restored rows are the same bytes.
constexpr size_t kFftRuns = 4;
constexpr uint64_t kBridgeBytes = uint64_t(128) << 20;
constexpr uint64_t kKeepOutRowBytes = 8192;

// Launch a pass at level k over the sets of the superblocks (2^(lo_k + K_k)
// rows) whose `weight` is nonzero, as at most kFftRuns runs of consecutive sets.
// `rows` (optional): rows read (IFFT) or written (reveal) per superblock, for
// the profiler's byte counts; else `weight` is that count.
void launch_runs(rs::PassArgs P, const Levels &lv, uint32_t k, int flags, const std::vector<uint64_t> &weight,
                 hipStream_t s, bool wr_weight, const std::vector<uint64_t> *rows = nullptr) {
    const uint32_t a = lv.lo[k];
    std::vector<std::pair<uint32_t, uint32_t>> runs;  // [begin, end) superblocks
    std::vector<uint64_t> w;
    for (uint32_t sb = 0; sb < weight.size(); ++sb) {
        if (!weight[sb]) continue;
        const uint64_t n = rows ? (*rows)[sb] : weight[sb];
        if (!runs.empty() && runs.back().second == sb) {
            runs.back().second = sb + 1;
            w.back() += n;
        } else {
            runs.push_back({sb, sb + 1});
            w.push_back(n);
        }
    }
    // a gap of fewer than kBridgeBytes of rows costs less to transform than a
    // launch of its own (measured: 32768:32768 x 1 KiB, 1 % loss, profiles/r01o)
    const uint64_t set_bytes = (uint64_t(P.packs) * 8) << lv.K[k];
    for (size_t i = 0; i + 1 < runs.size();) {
        if (uint64_t(runs[i + 1].first - runs[i].second) * set_bytes << a < kBridgeBytes) {
            runs[i].second = runs[i + 1].second;
            w[i] += w[i + 1];
            runs.erase(runs.begin() + i + 1);
            w.erase(w.begin() + i + 1);
        } else {
            ++i;
        }
    }
    while (runs.size() > kFftRuns) {
        size_t j = 0;  // bridge the smallest gap: runs j and j + 1
        for (size_t i = 1; i + 1 < runs.size(); ++i)
            if (runs[i + 1].first - runs[i].second < runs[j + 1].first - runs[j].second) j = i;
        runs[j].second = runs[j + 1].second;
        w[j] += w[j + 1];
        runs.erase(runs.begin() + j + 1);
        w.erase(w.begin() + j + 1);
    }
    for (size_t i = 0; i < runs.size(); ++i) {
        P.set_base = runs[i].first << a;
        launch(int(lv.K[k]), flags, P, (runs[i].second - runs[i].first) << a, a, s, wr_weight ? 0 : w[i],
               wr_weight ? w[i] : 0);
    }
}

// Rows r of [r_begin, r_end) with st[r] == want, counted per 2^sb_log-row
// superblock (std::count over each block's bytes: vectorised; this runs on the
// host for every decode, ahead of launches that take ~100 us for 2^16 rows).
std::vector<uint64_t> count_per_block(const std::vector<uint8_t> &st, uint32_t nd, uint32_t sb_log, uint32_t r_begin,
                                      uint32_t r_end, uint8_t want) {
    std::vector<uint64_t> c(nd >> sb_log, 0);
    r_end = std::min(r_end, nd);
    for (uint32_t sb = 0; sb < c.size(); ++sb) {
        const uint32_t r0 = std::max(sb << sb_log, r_begin), r1 = std::min((sb + 1) << sb_log, r_end);
        if (r0 < r1) c[sb] = uint64_t(std::count(st.data() + r0, st.data() + r1, want));
    }
    return c;
}

void fft_pass_pruned(rs::PassArgs P, const Levels &lv, uint32_t k, uint32_t nd, const std::vector<uint8_t> &st,
                     const rs::RowMap &out, hipStream_t s) {
    launch_runs(P, lv, k, rs::kFft, count_per_block(st, nd, lv.lo[k] + lv.K[k], out.row_begin, out.row_end, 1), s,
                true);
}

// Decode (rate_high.rs:172-254 / rate_low.rs:172-254).  Only missing original
// rows of `restored` are written.
//
// Multi-level formal derivative (DESIGN.md "Formal derivative across passes"):
// with X_k the IFFT output after levels 0..k and P_(k) the derivative terms of
// level k's bits,  U = F_top(P_(top) X_top),  V_{m-2} = F_{m-2}((I + P_(m-2)) X_{m-2} + U),
// V_k = F_k(P_(k) X_k + V_{k+1}) for k < m-2, and V_0 is FFT(derivative(IFFT)).
void decode_dev(rs_context *ctx, Workspace &ws, bool high, const Geom &g, uint64_t N, uint64_t M,
                const uint8_t *orig, const uint8_t *orig_present, const uint8_t *rec, const uint8_t *rec_present,
                uint8_t *restored, hipStream_t s) {
    const uint32_t chunk = uint32_t(high ? next_pow2(M) : next_pow2(N));
    const uint32_t end = uint32_t(chunk + (high ? N : M));
    uint32_t nd = uint32_t(next_pow2(end)), u = ilog2(nd);
    // Decodes of 16..64 work rows run the column kernel's smallest transform,
    // 2^kMonoMinL rows: the rows past `end` are neither received nor erased
    // (zero, as past 2^u), and any power of two >= end decodes the same bytes
    // (eval_poly folds exactly onto it).  32:32 x 1 KiB decode
    // 7.8 -> 6.0 us against the single fused pass; below 16 rows the pass is
    // faster (1:1 4.8 vs 5.7 us; profiles/r04a/pad_small.txt).  RS_MI355X_PAD_SMALL=0: off
    if (ctx->pad_small && nd >= 16 && nd < (1u << kMonoMinL) && ctx->mono && g.packs <= ctx->mono_max_packs) {
        nd = 1u << kMonoMinL;
        u = kMonoMinL;
    }
    // erasure vector + received flags per work row
    std::vector<uint8_t> &st = ws.h_state;
    st.assign(nd, 0);
    if (high) {
        for (uint32_t r = 0; r < M; ++r) st[r] = rec_present[r] ? 2 : 1;
        for (uint32_t r = uint32_t(M); r < chunk; ++r) st[r] = 1;
        for (uint32_t r = chunk; r < end; ++r) st[r] = orig_present[r - chunk] ? 2 : 1;
    } else {
        for (uint32_t r = 0; r < N; ++r) st[r] = orig_present[r] ? 2 : 1;
        for (uint32_t r = chunk; r < end; ++r) st[r] = rec_present[r - chunk] ? 2 : 1;
    }
    uint64_t received = 0, missing = 0;
    for (uint32_t r = 0; r < nd; ++r) received += st[r] == 2;
    for (uint64_t i = 0; i < N; ++i) missing += !orig_present[i];
    const rs::RowMap rec_map{rec, g.rec(), high ? 0u : chunk, high ? uint32_t(M) : end};
    const rs::RowMap orig_map{orig, g.orig(), high ? chunk : 0u, high ? end : uint32_t(N)};
    const rs::RowMap out_map{restored, g.out(), orig_map.row_begin, orig_map.row_end};
    const bool mono = use_mono(ctx, u, g, 1);
    const bool fused = mono && rs::mono_staged(int(u), 1) && nd <= rs::kMonoFusedRows;
    if (g.stripes > 1 && !fused) {  // batch: one stripe after another
        Geom g1 = g;
        g1.stripes = 1;
        for (uint32_t b = 0; b < g.stripes; ++b)
            decode_dev(ctx, ws, high, g1, N, M, orig + b * g.orig_bstride, orig_present, rec + b * g.rec_bstride,
                       rec_present, restored + b * g.out_bstride, s);
        return;
    }
    if (fused) {
        // one launch: every column workgroup evaluates eval_poly itself
        rs::MonoArgs Mo = mono_args(ctx, u, g, true, true);
        Mo.src[0] = rec_map;
        Mo.src_bstride[0] = g.rec_bstride;
        Mo.src[1] = orig_map;
        Mo.src_bstride[1] = g.orig_bstride;
        Mo.nsrc = 2;
        // the destination map narrowed to the span of the erased originals: the
        // waves holding no row of it after the FFT's last remap stop there
        // (wave_stores), so at 1 % loss (11 restored rows of 2^11) one wave of 16
        // runs the FFT's last in-wave layers, the reveal multiply and the stores
        // instead of the 8 of the restored half (VALU accounting,
        // profiles/r06c/valu_account.txt); present rows are never written either way
        {
            uint32_t lo = out_map.row_end, hi = out_map.row_begin;
            for (uint32_t r = out_map.row_begin; r < out_map.row_end; ++r)
                if (st[r] == 1) lo = std::min(lo, r), hi = r + 1;
            Mo.dst = lo < hi ? rs::RowMap{out_map.base + uint64_t(lo - out_map.row_begin) * out_map.stride,
                                          out_map.stride, lo, hi}
                             : out_map;
        }
        Mo.dst_bstride = g.out_bstride;
        Mo.fused_eval = 1;
        Mo.low_rate = high ? 0 : 1;
        Mo.end = end;
        Mo.lw0 = ctx->lw0;
        Mo.lw_fold = ctx->d_lwfold + (nd - 1);
        for (uint32_t r = 0; r < nd; ++r) {
            Mo.erased[r >> 5] |= uint32_t(st[r] == 1) << (r & 31);
            Mo.received[r >> 5] |= uint32_t(st[r] == 2) << (r & 31);
        }
        // (2^9 rows: the plain plan is faster, 256:256 x 1 KiB 8.3-8.8 -> 7.7 us;
        // equal at 2^10, the split plan faster at 2^11: profiles/r04a/split_ab.txt)
        if (ctx->split && rs::mono_split(int(u)) && u >= 10) {
            // split plan: every restored row in one half of the work rows
            bool lower = false, upper = false;
            for (uint32_t r = out_map.row_begin; r < out_map.row_end; ++r)
                if (st[r] == 1) (r < nd / 2 ? lower : upper) = true;
            if (!(lower && upper)) {
                Mo.split = 1;
                Mo.out_half = upper ? 1 : 0;
            }
        }
        launch_mono(rs::kMonoDecode, u, Mo, s, (received + missing) * uint64_t(g.packs) * 8 * g.stripes);
        return;
    }
    if (!mono && nd <= rs::kPassEvalRows && levels(u, max_k_dec(u, g.packs)).m == 1) {
        // one launch: the single pass evaluates eval_poly itself (rs_kernels.hip
        // pass_eval_poly), the erasure state in its arguments
        rs::PassArgs A = base_args(ctx, g, nd);
        A.src[0] = rec_map;
        A.src[1] = orig_map;
        A.nsrc = 2;
        A.load_scale = 1;
        A.fd_mode = 2;
        A.dst = out_map;
        A.reveal = 1;
        A.fused_eval = 1;
        A.ev_low_rate = high ? 0 : 1;
        A.ev_end = end;
        A.ev_lw0 = ctx->lw0;
        A.ev_lw_fold = ctx->d_lwfold + (nd - 1);
        for (uint32_t r = 0; r < nd; ++r) {
            A.ev_erased[r >> 5] |= uint32_t(st[r] == 1) << (r & 31);
            A.ev_received[r >> 5] |= uint32_t(st[r] == 2) << (r & 31);
        }
        run_level(A, levels(u, max_k_dec(u, g.packs)), 0, rs::kIfft | rs::kFft, nd, s, received, missing);
        return;
    }
    uint32_t *d_rowinfo = static_cast<uint32_t *>(ws.rowinfo.get(size_t(nd) * 4));
    rs::EvalArgs E;
    E.u = u;
    E.low_rate = high ? 0 : 1;
    E.end = end;
    E.lw0 = ctx->lw0;
    E.lw_fold = ctx->d_lwfold + (nd - 1);
    E.rowinfo = d_rowinfo;
    if (nd <= rs::kEvalInlineRows) {
        // the erasure state rides in the kernel arguments: no copy
        for (uint32_t r = 0; r < nd; ++r) {
            E.erased[r >> 5] |= uint32_t(st[r] == 1) << (r & 31);
            E.received[r >> 5] |= uint32_t(st[r] == 2) << (r & 31);
        }
    } else {
        uint8_t *d_state = static_cast<uint8_t *>(ws.state.get(nd));
        uint8_t *h = ws.h_state_pinned.get(nd);
        std::memcpy(h, st.data(), nd);
        check(hipMemcpyAsync(d_state, h, nd, hipMemcpyHostToDevice, s));
        ws.h_state_pinned.copied_on(s);
        E.state = d_state;
    }
    hipEvent_t ev = nullptr;
    if (t_prof_ctx) prof_begin(s, &ev);
    check(rs::launch_eval_poly(E, s));
    if (t_prof_ctx) prof_end(s, ev, "k_eval_poly", uint64_t(nd) * 5);

    if (use_half(ctx, u, g, 1)) {  // IFFT and FFT skew 0 (rate_high.rs:213-245)
        uint32_t in_h = 0, out_h = 0;
        for (uint32_t r = 0; r < nd; ++r) in_h |= uint32_t(st[r] == 2) << (r >> 11);
        for (uint32_t r = out_map.row_begin; r < out_map.row_end; ++r) out_h |= uint32_t(st[r] == 1) << (r >> 11);
        const rs::RowMap src[2] = {rec_map, orig_map};
        half_split(ctx, ws, g, true, 0, 0, src, 2, out_map, d_rowinfo, in_h, out_h, received, missing, s);
        return;
    }
    rs::PassArgs A = base_args(ctx, g, nd);
    A.rowinfo = d_rowinfo;
    if (mono) {
        rs::MonoArgs Mo = mono_args(ctx, u, g, false);
        Mo.src[0] = rec_map;
        Mo.src[1] = orig_map;
        Mo.nsrc = 2;
        Mo.dst = out_map;
        Mo.rowinfo = d_rowinfo;
        launch_mono(rs::kMonoDecode, u, Mo, s, (received + missing) * uint64_t(g.packs) * 8);
        return;
    }
    const Levels lv = levels(u, max_k_dec(u, g.packs));
    if (lv.m == 1) {
        A.src[0] = rec_map;
        A.src[1] = orig_map;
        A.nsrc = 2;
        A.load_scale = 1;
        A.fd_mode = 2;
        A.dst = out_map;
        A.reveal = 1;
        run_level(A, lv, 0, rs::kIfft | rs::kFft, nd, s, received, missing);
        return;
    }
    uint8_t *X[3];
    for (uint32_t k = 0; k + 1 < lv.m; ++k) X[k] = static_cast<uint8_t *>(ws.buf[k].get(size_t(nd) * g.stride));
    uint8_t *U = static_cast<uint8_t *>(ws.buf[3].get(size_t(nd) * g.stride));
    A.work_stride = g.stride;
    // Blocks of 2^G rows, G = the top level's lowest bit (2^K_top <= 256 blocks):
    // a block with no received row has a zero IFFT below the top level (not
    // computed; read as zero), and the passes from the top down store U only
    // for the blocks the pruned FFT passes read
    const uint32_t G = lv.lo[lv.m - 1];
    // A/B measurement switch: 1 = no block masks, 2 = no IFFT-pass pruning (store masks only)
    static const int prune_mode = getenv("RS_MI355X_DECODE_PRUNE") ? atoi(getenv("RS_MI355X_DECODE_PRUNE")) : 0;
    const bool masks = prune_mode != 1 && (nd >> G) <= 256;
    const bool prune_ifft = masks && prune_mode != 2;
    std::vector<uint64_t> recv_blk;
    bool skips = false;  // some block's IFFT is skipped
    if (masks) {
        recv_blk = count_per_block(st, nd, G, 0, nd, 2);
        if (prune_ifft) {  // the blocks the IFFT passes launch: runs as launch_runs bridges them
            const uint64_t blk_bytes = (uint64_t(g.packs) * 8) << G;
            std::vector<std::pair<uint32_t, uint32_t>> runs;
            for (uint32_t b = 0; b < recv_blk.size(); ++b) {
                if (!recv_blk[b]) continue;
                if (!runs.empty() && (b - runs.back().second) * blk_bytes < kBridgeBytes) runs.back().second = b + 1;
                else runs.push_back({b, b + 1});
            }
            std::vector<uint64_t> live(recv_blk.size(), 0);
            for (size_t i = 0; i < runs.size(); ++i) {
                // beyond kFftRuns runs the launcher bridges the smallest gaps: keep those blocks live
                const uint32_t end = i + 1 < runs.size() && runs.size() > kFftRuns ? runs[i + 1].first : runs[i].second;
                for (uint32_t b = runs[i].first; b < end; ++b) live[b] = 1;
            }
            for (uint32_t b = 0; b < recv_blk.size(); ++b) {
                if (!live[b]) {
                    A.zero_in[b >> 6] |= 1ull << (b & 63);
                    skips = true;
                }
                recv_blk[b] = live[b];
            }
        }
        // U stores are skipped per row only where rows are long enough for the
        // saved write to outweigh the per-row test (measured, profiles/r01o)
        if (uint64_t(g.packs) * 8 >= kKeepOutRowBytes) {
            const std::vector<uint64_t> keep_blk = count_per_block(st, nd, G, out_map.row_begin, out_map.row_end, 1);
            for (uint32_t b = 0; b < keep_blk.size(); ++b)
                if (!keep_blk[b]) A.keep_out[b >> 6] &= ~(1ull << (b & 63));
        }
        A.blk_shift = G;
    }
    const bool top_masks = masks && (skips || uint64_t(g.packs) * 8 >= kKeepOutRowBytes);
    for (uint32_t k = 0; k + 1 < lv.m; ++k) {  // scale received rows (level 0), IFFT low levels
        rs::PassArgs P = A;
        if (k == 0) {
            P.src[0] = rec_map;
            P.src[1] = orig_map;
            P.nsrc = 2;
            P.load_scale = 1;
        } else {
            P.work_in = X[k - 1];
        }
        P.work_out = X[k];
        if (prune_ifft) {  // level-k superblocks inside blocks with received rows
            const uint32_t sb_log = lv.lo[k] + lv.K[k];
            std::vector<uint64_t> w(nd >> sb_log), rd(nd >> sb_log, 0);
            for (uint32_t sb = 0; sb < w.size(); ++sb) w[sb] = recv_blk[(sb << sb_log) >> G];
            if (k == 0 && t_prof_ctx) rd = count_per_block(st, nd, sb_log, 0, nd, 2);  // profiler bytes only
            launch_runs(P, lv, k, rs::kIfft, w, s, false, &rd);
        } else {
            run_level(P, lv, k, rs::kIfft, nd, s, k == 0 ? received : 0, 0);
        }
    }
    rs::PassArgs T = A;  // top: IFFT, its derivative terms, FFT -> U
    T.work_in = X[lv.m - 2];
    T.fd_mode = 1;
    T.work_out = U;
    T.blk_masks = top_masks ? 1 : 0;
    // its butterflies pruned by block (rs_kernels.hip Prune): the IFFT skips groups of
    // zero-input blocks, the FFT groups that feed no block with restored rows
    // (RS_MI355X_BFLY_PRUNE=0: off, A/B)
    static const bool bfly_prune = !getenv("RS_MI355X_BFLY_PRUNE") || getenv("RS_MI355X_BFLY_PRUNE")[0] != '0';
    if (bfly_prune && masks && lv.K[lv.m - 1] <= 6) {
        const std::vector<uint64_t> need = count_per_block(st, nd, G, out_map.row_begin, out_map.row_end, 1);
        T.bfly_prune = 1;
        T.zin_local = top_masks ? A.zero_in[0] : 0;
        T.need_local = 0;
        for (uint32_t b = 0; b < need.size(); ++b)
            if (need[b]) T.need_local |= 1ull << b;
    }
    run_level(T, lv, lv.m - 1, rs::kIfft | rs::kFft, nd, s);
    A.blk_masks = skips ? 1 : 0;  // the passes below the top read X[k]: zero blocks load as zero
    A.blk_uniform = 1;
    for (int k = int(lv.m) - 2; k >= 0; --k) {  // V_k, last one revealed
        rs::PassArgs P = A;
        P.work_in = X[k];
        P.fd_mode = k == int(lv.m) - 2 ? 2 : 1;
        P.xor_in = U;
        if (k == 0) {
            P.dst = out_map;
            P.reveal = 1;
        } else {
            P.work_out = U;
        }
        fft_pass_pruned(P, lv, uint32_t(k), nd, st, out_map, s);
    }
}

const char *hip_msg(hipError_t e) { return hipGetErrorString(e); }

}  // namespace

// ===========================================================================
// encoder / decoder objects

// Host staging of the object API: pinned (the copies to and from the device
// run asynchronously at the link's rate, with no bounce through a pageable
// buffer), portable (any device's copies may use it: a work hand-off moves it
// to a context on another GPU), grown monotonically, contents not kept.
struct HostStage {
    uint8_t *p = nullptr;
    size_t cap = 0;
    HostStage() = default;
    HostStage(const HostStage &) = delete;
    HostStage &operator=(const HostStage &) = delete;
    uint8_t *get(size_t bytes) {
        if (bytes > cap) {
            if (p) check(hipHostFree(p));
            p = nullptr;
            cap = 0;
            void *q = nullptr;
            check(hipHostMalloc(&q, bytes ? bytes : 1, hipHostMallocPortable));
            p = static_cast<uint8_t *>(q);
            cap = bytes;
        }
        return p;
    }
    void swap(HostStage &o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
    }
    ~HostStage() {
        if (p) (void)hipHostFree(p);
    }
};
// The stream an encoder's / decoder's copies and kernels run on (created on
// the object's device at its first encode / decode).
struct ObjStream {
    hipStream_t s = nullptr;
    ObjStream() = default;
    ObjStream(const ObjStream &) = delete;
    ObjStream &operator=(const ObjStream &) = delete;
    hipStream_t get() {  // on the object's device
        if (!s) check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        return s;
    }
    void swap(ObjStream &o) { std::swap(s, o.s); }
    ~ObjStream() {
        if (s) (void)hipStreamDestroy(s);
    }
};

struct rs_encoder {
    rs_context *ctx;
    rs_rate rate;
    bool high = true;
    uint64_t N = 0, M = 0, S = 0, row = 0, received = 0;
    bool has_result = false;
    HostStage h_orig, h_rec;      // padded rows (64-byte blocks, shards.rs:38-59)
    std::vector<uint8_t> h_tail;  // unpadded result when S % 64 != 0
    DevBuf d_orig, d_rec;
    Workspace ws;
    ObjStream st;
};

struct rs_decoder {
    rs_context *ctx;
    rs_rate rate;
    bool high = true;
    uint64_t N = 0, M = 0, S = 0, row = 0;
    uint64_t orig_received = 0, rec_received = 0;
    bool has_result = false, decoded = false;
    std::vector<uint8_t> orig_present, rec_present;
    HostStage h_orig, h_rec, h_out;  // padded rows
    std::vector<uint8_t> h_tail;     // unpadded restored rows when S % 64 != 0
    DevBuf d_orig, d_rec, d_out;
    Workspace ws;
    ObjStream st;
};

// EncoderWork / DecoderWork (src/rate.rs:129-139): the buffers of an encoder /
// decoder handed from one object to the next (any rate, any shape).  The
// device buffers, the stream (and the pinned staging's event) belong to the
// device of the context that made them (`device`): swap_host moves only the
// host buffers, for a context on another device (device memory of GPU0 must
// not back GPU1's kernels).
struct rs_encoder_work {
    int device = -1;
    HostStage h_orig, h_rec;
    std::vector<uint8_t> h_tail;
    DevBuf d_orig, d_rec;
    Workspace ws;
    ObjStream st;
    void swap_host(rs_encoder &e) {
        h_orig.swap(e.h_orig);
        h_rec.swap(e.h_rec);
        h_tail.swap(e.h_tail);
    }
    void swap(rs_encoder &e) {
        swap_host(e);
        d_orig.swap(e.d_orig);
        d_rec.swap(e.d_rec);
        ws.swap(e.ws);
        st.swap(e.st);
    }
};
struct rs_decoder_work {
    int device = -1;
    std::vector<uint8_t> orig_present, rec_present, h_tail;
    HostStage h_orig, h_rec, h_out;
    DevBuf d_orig, d_rec, d_out;
    Workspace ws;
    ObjStream st;
    void swap_host(rs_decoder &d) {
        orig_present.swap(d.orig_present);
        rec_present.swap(d.rec_present);
        h_orig.swap(d.h_orig);
        h_rec.swap(d.h_rec);
        h_out.swap(d.h_out);
        h_tail.swap(d.h_tail);
    }
    void swap(rs_decoder &d) {
        swap_host(d);
        d_orig.swap(d.d_orig);
        d_rec.swap(d.d_rec);
        d_out.swap(d.d_out);
        ws.swap(d.ws);
        st.swap(d.st);
    }
};

namespace {

// tail re-pack of a shard into padded 64-byte blocks (shards.rs:38-59)
void insert_row(uint8_t *dst, const uint8_t *src, uint64_t S) {
    const uint64_t whole = S / 64, tail = S % 64;
    std::memcpy(dst, src, whole * 64);
    if (tail) {
        uint8_t *blk = dst + whole * 64;
        std::memset(blk, 0, 64);
        std::memcpy(blk, src + whole * 64, tail / 2);
        std::memcpy(blk + 32, src + whole * 64 + tail / 2, tail / 2);
    }
}
// undo (shards.rs:62-74)
void extract_row(uint8_t *dst, const uint8_t *src, uint64_t S) {
    const uint64_t whole = S / 64, tail = S % 64;
    std::memcpy(dst, src, whole * 64);
    if (tail) {
        std::memcpy(dst + whole * 64, src + whole * 64, tail / 2);
        std::memcpy(dst + whole * 64 + tail / 2, src + whole * 64 + 32, tail / 2);
    }
}

template <typename F>
rs_status guarded(rs_error *err, F &&f) {
    try {
        return f();
    } catch (const DevError &d) {
        g_last_error = hip_msg(d.e);
        return set_err(err, RS_ERR_DEVICE);
    } catch (const std::bad_alloc &) {
        g_last_error = "host allocation failed";
        return set_err(err, RS_ERR_DEVICE);
    }
}

rs_status encoder_configure(rs_encoder *e, uint64_t N, uint64_t M, uint64_t S, rs_error *err) {
    const int high = resolve(e->rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    e->high = high;
    e->N = N, e->M = M, e->S = S;
    e->row = round_up(S, 64);
    e->received = 0;
    e->has_result = false;
    // pinned staging of the padded originals, written by add_original_shard
    return guarded(err, [&]() -> rs_status {
        e->h_orig.get(N * e->row);
        return set_err(err, RS_OK);
    });
}

rs_status decoder_configure(rs_decoder *d, uint64_t N, uint64_t M, uint64_t S, rs_error *err) {
    const int high = resolve(d->rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    d->high = high;
    d->N = N, d->M = M, d->S = S;
    d->row = round_up(S, 64);
    d->orig_received = d->rec_received = 0;
    d->has_result = d->decoded = false;
    d->orig_present.assign(N, 0);
    d->rec_present.assign(M, 0);
    return guarded(err, [&]() -> rs_status {
        d->h_orig.get(N * d->row);
        d->h_rec.get(M * d->row);
        return set_err(err, RS_OK);
    });
}

void encoder_drop_result(rs_encoder *e) {
    if (e->has_result) {
        e->has_result = false;
        e->received = 0;  // EncoderResult::drop -> reset_received (encoder_result.rs:48-52)
    }
}
void decoder_drop_result(rs_decoder *d) {
    if (d->has_result) {
        d->has_result = d->decoded = false;  // DecoderResult::drop (decoder_result.rs:44-48)
        d->orig_received = d->rec_received = 0;
        std::fill(d->orig_present.begin(), d->orig_present.end(), 0);
        std::fill(d->rec_present.begin(), d->rec_present.end(), 0);
    }
}

}  // namespace

extern "C" {

const char *rs_last_device_error(void) { return g_last_error.c_str(); }
const char *rs_version(void) { return "rs-mi355x 0.1.0 (gfx950)"; }

rs_status rs_context_create(int device, rs_context **out) {
    if (!out) return RS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    auto *ctx = new rs_context;
    ctx->device = device;
    rs_status st = guarded(nullptr, [&]() -> rs_status {
        DeviceGuard dg(device);
        const rs::GfTables &T = rs::tables();
        check(hipMalloc(&ctx->d_tw, T.perm_by_skew.size() * 4));
        check(hipMalloc(&ctx->d_lut, T.perm_by_log.size() * 4));
        // lw_fold's 2^u-entry segment starts at entry 2^u - 1 (gf_tables.hpp); one
        // leading pad entry puts every segment of 2 or more entries on a 4-byte
        // boundary (the column kernel reads a thread's pair as one dword)
        check(hipMalloc(&ctx->d_lwfold_base, (T.lw_fold.size() + 1) * 2));
        ctx->d_lwfold = ctx->d_lwfold_base + 1;
        check(hipMemcpy(ctx->d_tw, T.perm_by_skew.data(), T.perm_by_skew.size() * 4, hipMemcpyHostToDevice));
        check(hipMemcpy(ctx->d_lut, T.perm_by_log.data(), T.perm_by_log.size() * 4, hipMemcpyHostToDevice));
        check(hipMemcpy(ctx->d_lwfold, T.lw_fold.data(), T.lw_fold.size() * 2, hipMemcpyHostToDevice));
        check(hipMalloc(&ctx->d_lut2, T.perm2_by_log.size() * 4));
        check(hipMemcpy(ctx->d_lut2, T.perm2_by_log.data(), T.perm2_by_log.size() * 4, hipMemcpyHostToDevice));
        ctx->lw0 = T.log_walsh[0];
        if (const char *pb = getenv("RS_MI355X_PASS_BASIS")) ctx->pass_basis = pb[0] == '1';
        if (ctx->pass_basis) pass_basis_tables(ctx);
        int cus = 0;
        check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        ctx->e2_max_packs = ctx->e2_default = cus > 1 ? uint32_t(cus) / 2 : 1u;
        if (const char *ln = getenv("RS_MI355X_LANE")) ctx->lane = ln[0] == '1';
        ctx->lane_default = ctx->lane;
        if (const char *hs = getenv("RS_MI355X_HALF")) ctx->half = hs[0] == '1';
        ctx->half_default = ctx->half;
        if (const char *qs = getenv("RS_MI355X_QUAD")) ctx->quad = qs[0] == '1';
        if (const char *cp = getenv("RS_MI355X_COPYIN_POOL")) ctx->copyin_pool = cp[0] == '1';
        ctx->quad_default = ctx->quad;
        if (const char *ck = getenv("RS_MI355X_CHUNKS")) {  // 0 off, 1 default routing, 2 every supported shape
            ctx->chunks = ck[0] != '0';
            ctx->chunks_forced = ck[0] == '2';
        }
        ctx->chunks_default = ctx->chunks;
        ctx->chunks_forced_default = ctx->chunks_forced;
        {  // top_table: skew index 2047 + 2048 j, both table formats
            std::vector<uint32_t> top(size_t(kTopTables) * (rs::kPermWords + rs::kPerm2Words));
            for (uint32_t j = 0; j < kTopTables; ++j) {
                const size_t idx = 2047 + 2048 * size_t(j);
                std::copy_n(&T.perm_by_skew[idx * rs::kPermWords], rs::kPermWords, &top[j * rs::kPermWords]);
                std::copy_n(&T.perm2_by_skew[idx * rs::kPerm2Words], rs::kPerm2Words,
                            &top[kTopTables * rs::kPermWords + j * rs::kPerm2Words]);
            }
            check(hipMalloc(&ctx->d_top, top.size() * 4));
            check(hipMemcpy(ctx->d_top, top.data(), top.size() * 4, hipMemcpyHostToDevice));
        }
        const char *psm = getenv("RS_MI355X_PAD_SMALL");
        if (psm) ctx->pad_small = psm[0] == '1';
        const char *nm = getenv("RS_MI355X_NO_MONO");
        ctx->mono = !(nm && nm[0] == '1');
        if (const char *mk = getenv("RS_MI355X_MAX_K")) {
            const unsigned long k = strtoul(mk, nullptr, 10);
            if (k >= 4 && k <= kMaxK) g_max_k = uint32_t(k);
        }
        const char *ns = getenv("RS_MI355X_NO_SPLIT");
        ctx->split = !(ns && ns[0] == '1');
        const char *ma = getenv("RS_MI355X_MONO_ALL");
        ctx->mono_all = ma && ma[0] == '1';
        if (const char *mp = getenv("RS_MI355X_MONO_MAX_PACKS")) ctx->mono_max_packs = uint32_t(strtoul(mp, nullptr, 10));
        if (const char *e2 = getenv("RS_MI355X_E2_MAX_PACKS"))  // also what rs_mono_enable resets to
            ctx->e2_max_packs = ctx->e2_default = uint32_t(strtoul(e2, nullptr, 10));
        if (const char *cp = getenv("RS_MI355X_CHUNK_PARALLEL"))  // "0" / "1"; anything else: automatic
            ctx->chunk_par = cp[0] == '1' && !cp[1] ? 1 : cp[0] == '0' && !cp[1] ? 0 : -1;
        // column-kernel twiddle images of every transform size, built now: a lazy
        // build inside an asynchronous call would stall the device with a
        // synchronous upload the first time a size is seen
        for (uint32_t L = kChunksMinL; L <= kMonoMaxL; ++L) mono_images(ctx, L);
        for (uint32_t L = kChunksMinL; L <= 11; ++L) mono_images(ctx, L, 2);
        for (uint32_t L = kChunksMinL; L <= (RS_MONO_BASIS ? 11u : 10u); ++L) basis_images(ctx, L);  // (k_lane: 8..10)
        for (uint32_t L = kChunksMinL; L <= 7; ++L) basis_images(ctx, L, 4);
        return RS_OK;
    });
    if (st != RS_OK) {
        rs_context_destroy(ctx);
        return st;
    }
    *out = ctx;
    return RS_OK;
}

void rs_context_destroy(rs_context *ctx) {
    if (!ctx) return;
    for (rs_encoder_work *w : ctx->enc_pool) rs_encoder_work_free(w);
    for (rs_decoder_work *w : ctx->dec_pool) rs_decoder_work_free(w);
    delete ctx->pipe;
    if (ctx->d_tw) (void)hipFree(ctx->d_tw);
    if (ctx->d_lut) (void)hipFree(ctx->d_lut);
    if (ctx->d_lut2) (void)hipFree(ctx->d_lut2);
    if (ctx->d_twb) (void)hipFree(ctx->d_twb);
    if (ctx->d_lutb) (void)hipFree(ctx->d_lutb);
    if (ctx->d_top) (void)hipFree(ctx->d_top);
    for (uint32_t *p : ctx->d_img2)
        if (p) (void)hipFree(p);
    for (uint32_t *p : ctx->d_imgb)
        if (p) (void)hipFree(p);
    for (uint32_t *p : ctx->d_imgb4)
        if (p) (void)hipFree(p);
    if (ctx->d_lwfold_base) (void)hipFree(ctx->d_lwfold_base);
    for (uint32_t *p : ctx->d_img)
        if (p) (void)hipFree(p);
    delete ctx;
}

int rs_use_high_rate(uint64_t N, uint64_t M) { return use_high_rate(N, M); }

int rs_supports(rs_rate rate, uint64_t N, uint64_t M) {
    if (rate == RS_RATE_HIGH) return high_supported(N, M);
    if (rate == RS_RATE_LOW) return low_supported(N, M);
    return use_high_rate(N, M) >= 0;
}

rs_status rs_validate(rs_rate rate, uint64_t N, uint64_t M, uint64_t S, rs_error *err) {
    if (resolve(rate, N, M, S, err) < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    return set_err(err, RS_OK);
}

uint64_t rs_encoder_work_count(rs_rate rate, uint64_t N, uint64_t M) {
    const int high = rate == RS_RATE_HIGH ? 1 : rate == RS_RATE_LOW ? 0 : use_high_rate(N, M);
    if (high < 0) return 0;
    return high ? round_up(N, next_pow2(M)) : round_up(M, next_pow2(N));
}

uint64_t rs_decoder_work_count(rs_rate rate, uint64_t N, uint64_t M) {
    const int high = rate == RS_RATE_HIGH ? 1 : rate == RS_RATE_LOW ? 0 : use_high_rate(N, M);
    if (high < 0) return 0;
    return high ? next_pow2(next_pow2(M) + N) : next_pow2(next_pow2(N) + M);
}

// ---- device-resident ------------------------------------------------------

namespace {
// any row stride that holds a shard (0 = shard_bytes); any device address:
// unaligned matrices go byte by byte (ShardFormat::io_bytes)
bool stride_ok(uint64_t stride, uint64_t S) { return stride == 0 || stride >= S; }
bool ptr_ok(const void *p) { return p != nullptr; }
}  // namespace

rs_status rs_encode_device_strided(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S,
                                   const void *d_orig, uint64_t orig_stride, void *d_rec, uint64_t rec_stride,
                                   void *stream, rs_error *err) {
    if (!ctx || !ptr_ok(d_orig) || !ptr_ok(d_rec)) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const int high = resolve(rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    if (!stride_ok(orig_stride, S) || !stride_ok(rec_stride, S)) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    return guarded(err, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        ProfScope prof(ctx);
        const Geom g = device_geom(S, orig_stride, rec_stride, 0, {d_orig, d_rec});
        auto s = static_cast<hipStream_t>(stream);
        StreamWs sw(ctx, s);
        if (high)
            encode_high(ctx, sw.w, g, N, M, static_cast<const uint8_t *>(d_orig), static_cast<uint8_t *>(d_rec), s);
        else
            encode_low(ctx, sw.w, g, N, M, static_cast<const uint8_t *>(d_orig), static_cast<uint8_t *>(d_rec), s);
        return set_err(err, RS_OK);
    });
}

rs_status rs_encode_device(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, const void *d_orig,
                           void *d_rec, void *stream, rs_error *err) {
    return rs_encode_device_strided(ctx, rate, N, M, S, d_orig, 0, d_rec, 0, stream, err);
}

rs_status rs_encode_device_batch(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, uint64_t stripes,
                                 const void *d_orig, uint64_t orig_stride, uint64_t orig_stripe_stride, void *d_rec,
                                 uint64_t rec_stride, uint64_t rec_stripe_stride, void *stream, rs_error *err) {
    if (!ctx || !ptr_ok(d_orig) || !ptr_ok(d_rec)) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const int high = resolve(rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    if (!stride_ok(orig_stride, S) || !stride_ok(rec_stride, S)) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const uint64_t orig_b = orig_stripe_stride ? orig_stripe_stride : N * (orig_stride ? orig_stride : S);
    const uint64_t rec_b = rec_stripe_stride ? rec_stripe_stride : M * (rec_stride ? rec_stride : S);
    if (stripes == 0) return set_err(err, RS_OK);
    return guarded(err, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        ProfScope prof(ctx);
        Geom g = device_geom(S, orig_stride, rec_stride, 0, {d_orig, d_rec});
        if ((orig_b | rec_b) % 4) g.fmt.io_bytes = 1, g.fmt.full_packs = uint32_t(S / 64 * 8), g.fmt.tail_h = uint32_t(S % 64 / 2);
        g.orig_bstride = orig_b;
        g.rec_bstride = rec_b;
        auto s = static_cast<hipStream_t>(stream);
        StreamWs sw(ctx, s);
        for (uint64_t b0 = 0; b0 < stripes; b0 += kMaxBatchStripes) {  // grid.y limit
            g.stripes = uint32_t(std::min<uint64_t>(kMaxBatchStripes, stripes - b0));
            const uint8_t *o = static_cast<const uint8_t *>(d_orig) + b0 * orig_b;
            uint8_t *r = static_cast<uint8_t *>(d_rec) + b0 * rec_b;
            if (high)
                encode_high(ctx, sw.w, g, N, M, o, r, s);
            else
                encode_low(ctx, sw.w, g, N, M, o, r, s);
        }
        return set_err(err, RS_OK);
    });
}

}  // extern "C"

// ---------------------------------------------------------------------------
// host-memory pipeline: the shard matrices live in host memory (pinned for
// full PCIe rate).  The byte axis is cut into column slices of whole 64-byte
// blocks (every op is column-wise, src/engine/utils.rs:35-43); slice k is
// copied in, coded and copied out on stream k % kStreams, so the copies of
// one slice overlap the kernels of its neighbours.

namespace {

rs_context::Pipe &pipe_of(rs_context *ctx) {
    if (!ctx->pipe) {
        auto *p = new rs_context::Pipe;
        for (hipStream_t &s : p->st) {
            hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            if (e != hipSuccess) {
                delete p;
                check(e);
            }
        }
        ctx->pipe = p;
    }
    return *ctx->pipe;
}

uint64_t slice_width(uint64_t S, uint32_t slices) {
    const uint64_t blocks = S / 64;
    const uint64_t k = std::max<uint64_t>(1, std::min<uint64_t>(slices ? slices : 1, blocks));
    return std::max<uint64_t>(64, (blocks + k - 1) / k * 64);  // S < 64: one slice (the tail)
}

// hipMemcpy2DAsync of the rows [r0, r1) where flag[r] == want, in runs.  With
// `span_ok` (the destination's other rows are scratch nobody reads), more than
// kCopyRuns runs go as one copy of the span from the first to the last wanted row:
// every copy costs ~10 us of latency, so scattered losses (hundreds of runs) would
// otherwise cost more than the bytes they skip.  Span copies carry absent rows in and
// present rows out, so they rely on two invariants: no decode route reads an absent
// row of d_orig / d_rec (erased rows load as zero, decode_dev), and only missing rows
// of an output staging are read back (restored_original); pinned by
// tests/test_gpu_parity.py::test_decode_ignores_absent_rows_and_stale_staging.
constexpr uint64_t kCopyRuns = 4;
void copy_rows(uint8_t *dst, const uint8_t *src, uint64_t pitch, uint64_t width, const uint8_t *flag, uint8_t want,
               uint64_t rows, hipMemcpyKind kind, hipStream_t s, bool span_ok = false) {
    if (flag && span_ok) {
        uint64_t runs = 0, first = rows, last = 0;
        for (uint64_t i = 0; i < rows; ++i)
            if ((flag[i] != 0) == (want != 0)) {
                runs += i == 0 || (flag[i - 1] != 0) != (want != 0);
                first = std::min(first, i);
                last = i;
            }
        if (runs > kCopyRuns) {
            copy_rows(dst + first * pitch, src + first * pitch, pitch, width, nullptr, 1, last + 1 - first, kind, s);
            return;
        }
    }
    uint64_t r = 0;
    while (r < rows) {
        if (flag && (flag[r] != 0) != (want != 0)) {
            ++r;
            continue;
        }
        uint64_t e = r + 1;
        while (e < rows && (!flag || (flag[e] != 0) == (want != 0))) ++e;
        if (width == pitch)  // whole rows: one linear copy of the run
            check(hipMemcpyAsync(dst + r * pitch, src + r * pitch, (e - r) * pitch, kind, s));
        else
            check(hipMemcpy2DAsync(dst + r * pitch, pitch, src + r * pitch, pitch, width, e - r, kind, s));
        r = e;
    }
}

}  // namespace

extern "C" {

void *rs_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void rs_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

rs_status rs_encode_host(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, const void *h_orig,
                         void *h_rec, uint32_t slices, rs_error *err) {
    if (!ctx || !h_orig || !h_rec) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const int high = resolve(rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    return guarded(err, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        ProfScope prof(ctx);
        auto &P = pipe_of(ctx);
        auto *d_o = static_cast<uint8_t *>(P.orig.get(N * S));
        auto *d_r = static_cast<uint8_t *>(P.rec.get(M * S));
        const auto *h_o = static_cast<const uint8_t *>(h_orig);
        auto *h_r = static_cast<uint8_t *>(h_rec);
        const uint64_t w = slice_width(S, slices);
        int k = 0;
        for (uint64_t a = 0; a < S; a += w, ++k) {
            const uint64_t b = std::min(S, a + w);
            hipStream_t s = P.st[k % rs_context::Pipe::kStreams];
            Workspace &ws = P.ws[k % rs_context::Pipe::kStreams];
            check(hipMemcpy2DAsync(d_o + a, S, h_o + a, S, b - a, N, hipMemcpyHostToDevice, s));
            const Geom g = device_geom(b - a, S, S, S, {d_o + a, d_r + a});
            if (high) encode_high(ctx, ws, g, N, M, d_o + a, d_r + a, s);
            else encode_low(ctx, ws, g, N, M, d_o + a, d_r + a, s);
            check(hipMemcpy2DAsync(h_r + a, S, d_r + a, S, b - a, M, hipMemcpyDeviceToHost, s));
        }
        for (hipStream_t s : P.st) check(hipStreamSynchronize(s));
        return set_err(err, RS_OK);
    });
}

rs_status rs_decode_host(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, const void *h_orig,
                         const uint8_t *orig_present, const void *h_rec, const uint8_t *rec_present,
                         void *h_restored, uint32_t slices, rs_error *err) {
    if (!ctx || !h_orig || !h_rec || !h_restored || !orig_present || !rec_present)
        return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const int high = resolve(rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    uint64_t have_o = 0, have_r = 0;
    for (uint64_t i = 0; i < N; ++i) have_o += orig_present[i] != 0;
    for (uint64_t i = 0; i < M; ++i) have_r += rec_present[i] != 0;
    if (have_o + have_r < N) {
        set_err(err, RS_ERR_NOT_ENOUGH_SHARDS);
        if (err) err->original_count = N, err->original_received_count = have_o, err->recovery_received_count = have_r;
        return RS_ERR_NOT_ENOUGH_SHARDS;
    }
    if (have_o == N) return set_err(err, RS_OK);
    return guarded(err, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        ProfScope prof(ctx);
        auto &P = pipe_of(ctx);
        auto *d_o = static_cast<uint8_t *>(P.orig.get(N * S));
        auto *d_r = static_cast<uint8_t *>(P.rec.get(M * S));
        auto *d_x = static_cast<uint8_t *>(P.out.get(N * S));
        const auto *h_o = static_cast<const uint8_t *>(h_orig);
        const auto *h_r = static_cast<const uint8_t *>(h_rec);
        auto *h_x = static_cast<uint8_t *>(h_restored);
        const uint64_t w = slice_width(S, slices);
        int k = 0;
        for (uint64_t a = 0; a < S; a += w, ++k) {
            const uint64_t b = std::min(S, a + w);
            hipStream_t s = P.st[k % rs_context::Pipe::kStreams];
            Workspace &ws = P.ws[k % rs_context::Pipe::kStreams];
            // only received rows travel in, only restored rows travel out
            // (absent rows of the device staging are scratch; the caller's h_restored is not)
            copy_rows(d_o + a, h_o + a, S, b - a, orig_present, 1, N, hipMemcpyHostToDevice, s, true);
            copy_rows(d_r + a, h_r + a, S, b - a, rec_present, 1, M, hipMemcpyHostToDevice, s, true);
            const Geom g = device_geom(b - a, S, S, S, {d_o + a, d_r + a, d_x + a});
            decode_dev(ctx, ws, high, g, N, M, d_o + a, orig_present, d_r + a, rec_present, d_x + a, s);
            copy_rows(h_x + a, d_x + a, S, b - a, orig_present, 0, N, hipMemcpyDeviceToHost, s);
        }
        for (hipStream_t s : P.st) check(hipStreamSynchronize(s));
        return set_err(err, RS_OK);
    });
}

rs_status rs_decode_device_strided(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S,
                                   const void *d_orig, uint64_t orig_stride, const uint8_t *orig_present,
                                   const void *d_rec, uint64_t rec_stride, const uint8_t *rec_present,
                                   void *d_restored, uint64_t restored_stride, void *stream, rs_error *err) {
    if (!ctx || !ptr_ok(d_orig) || !ptr_ok(d_rec) || !ptr_ok(d_restored) || !orig_present || !rec_present)
        return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const int high = resolve(rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    if (!stride_ok(orig_stride, S) || !stride_ok(rec_stride, S) || !stride_ok(restored_stride, S))
        return set_err(err, RS_ERR_INVALID_ARGUMENT);
    uint64_t have_o = 0, have_r = 0;
    for (uint64_t i = 0; i < N; ++i) have_o += orig_present[i] != 0;
    for (uint64_t i = 0; i < M; ++i) have_r += rec_present[i] != 0;
    if (have_o + have_r < N) {
        set_err(err, RS_ERR_NOT_ENOUGH_SHARDS);
        if (err) err->original_count = N, err->original_received_count = have_o, err->recovery_received_count = have_r;
        return RS_ERR_NOT_ENOUGH_SHARDS;
    }
    if (have_o == N) return set_err(err, RS_OK);
    return guarded(err, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        ProfScope prof(ctx);
        const Geom g = device_geom(S, orig_stride, rec_stride, restored_stride, {d_orig, d_rec, d_restored});
        StreamWs sw(ctx, static_cast<hipStream_t>(stream));
        decode_dev(ctx, sw.w, high, g, N, M, static_cast<const uint8_t *>(d_orig), orig_present,
                   static_cast<const uint8_t *>(d_rec), rec_present, static_cast<uint8_t *>(d_restored),
                   static_cast<hipStream_t>(stream));
        return set_err(err, RS_OK);
    });
}

rs_status rs_decode_device(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, const void *d_orig,
                           const uint8_t *orig_present, const void *d_rec, const uint8_t *rec_present,
                           void *d_restored, void *stream, rs_error *err) {
    return rs_decode_device_strided(ctx, rate, N, M, S, d_orig, 0, orig_present, d_rec, 0, rec_present, d_restored,
                                    0, stream, err);
}

rs_status rs_decode_device_batch(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, uint64_t stripes,
                                 const void *d_orig, uint64_t orig_stride, uint64_t orig_stripe_stride,
                                 const uint8_t *orig_present, const void *d_rec, uint64_t rec_stride,
                                 uint64_t rec_stripe_stride, const uint8_t *rec_present, void *d_restored,
                                 uint64_t restored_stride, uint64_t restored_stripe_stride, void *stream,
                                 rs_error *err) {
    if (!ctx || !ptr_ok(d_orig) || !ptr_ok(d_rec) || !ptr_ok(d_restored) || !orig_present || !rec_present)
        return set_err(err, RS_ERR_INVALID_ARGUMENT);
    const int high = resolve(rate, N, M, S, err);
    if (high < 0) return rs_status(err ? err->code : RS_ERR_UNSUPPORTED_SHARD_COUNT);
    if (!stride_ok(orig_stride, S) || !stride_ok(rec_stride, S) || !stride_ok(restored_stride, S))
        return set_err(err, RS_ERR_INVALID_ARGUMENT);
    uint64_t have_o = 0, have_r = 0;
    for (uint64_t i = 0; i < N; ++i) have_o += orig_present[i] != 0;
    for (uint64_t i = 0; i < M; ++i) have_r += rec_present[i] != 0;
    if (have_o + have_r < N) {
        set_err(err, RS_ERR_NOT_ENOUGH_SHARDS);
        if (err) err->original_count = N, err->original_received_count = have_o, err->recovery_received_count = have_r;
        return RS_ERR_NOT_ENOUGH_SHARDS;
    }
    if (have_o == N || stripes == 0) return set_err(err, RS_OK);
    return guarded(err, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        ProfScope prof(ctx);
        Geom g = device_geom(S, orig_stride, rec_stride, restored_stride, {d_orig, d_rec, d_restored});
        g.orig_bstride = orig_stripe_stride ? orig_stripe_stride : N * g.orig();
        g.rec_bstride = rec_stripe_stride ? rec_stripe_stride : M * g.rec();
        g.out_bstride = restored_stripe_stride ? restored_stripe_stride : N * g.out();
        if ((g.orig_bstride | g.rec_bstride | g.out_bstride) % 4)
            g.fmt.io_bytes = 1, g.fmt.full_packs = uint32_t(S / 64 * 8), g.fmt.tail_h = uint32_t(S % 64 / 2);
        StreamWs sw(ctx, static_cast<hipStream_t>(stream));
        for (uint64_t b0 = 0; b0 < stripes; b0 += kMaxBatchStripes) {  // grid.y limit
            g.stripes = uint32_t(std::min<uint64_t>(kMaxBatchStripes, stripes - b0));
            decode_dev(ctx, sw.w, high, g, N, M,
                       static_cast<const uint8_t *>(d_orig) + b0 * g.orig_bstride,
                       orig_present, static_cast<const uint8_t *>(d_rec) + b0 * g.rec_bstride, rec_present,
                       static_cast<uint8_t *>(d_restored) + b0 * g.out_bstride, static_cast<hipStream_t>(stream));
        }
        return set_err(err, RS_OK);
    });
}

// ---- encoder ----------------------------------------------------------------

rs_status rs_encoder_new(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, rs_encoder **out,
                         rs_error *err) {
    return rs_encoder_new_with_work(ctx, rate, N, M, S, nullptr, out, err);
}

rs_status rs_encoder_new_with_work(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S,
                                   rs_encoder_work *work, rs_encoder **out, rs_error *err) {
    std::unique_ptr<rs_encoder_work> w(work);  // consumed in every case (moved into `new`, rate.rs:133-139)
    if (!ctx || !out) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    *out = nullptr;
    auto *e = new rs_encoder;
    e->ctx = ctx;
    e->rate = rate;
    if (w) {
        if (w->device == ctx->device) w->swap(*e);
        else w->swap_host(*e);  // device buffers of another device: freed with w
    }
    const rs_status st = encoder_configure(e, N, M, S, err);
    if (st != RS_OK) {
        delete e;
        return st;
    }
    *out = e;
    return RS_OK;
}

rs_status rs_encoder_reset(rs_encoder *e, uint64_t N, uint64_t M, uint64_t S, rs_error *err) {
    if (!e) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    e->has_result = false;
    return encoder_configure(e, N, M, S, err);
}

rs_status rs_encoder_add_original_shard(rs_encoder *e, const uint8_t *shard, uint64_t len, rs_error *err) {
    if (!e || (!shard && len)) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    encoder_drop_result(e);
    if (e->received == e->N) {  // encoder_work.rs:56-59
        set_err(err, RS_ERR_TOO_MANY_ORIGINAL_SHARDS);
        if (err) err->original_count = e->N;
        return RS_ERR_TOO_MANY_ORIGINAL_SHARDS;
    }
    if (len != e->S) {  // encoder_work.rs:60-64
        set_err(err, RS_ERR_DIFFERENT_SHARD_SIZE);
        if (err) err->shard_bytes = e->S, err->got = len;
        return RS_ERR_DIFFERENT_SHARD_SIZE;
    }
    insert_row(e->h_orig.p + e->received * e->row, shard, e->S);
    ++e->received;
    return set_err(err, RS_OK);
}

rs_status rs_encoder_encode(rs_encoder *e, rs_error *err) {
    if (!e) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    if (e->has_result) return set_err(err, RS_OK);
    if (e->received != e->N) {  // encoder_work.rs:75-86
        set_err(err, RS_ERR_TOO_FEW_ORIGINAL_SHARDS);
        if (err) err->original_count = e->N, err->original_received_count = e->received;
        return RS_ERR_TOO_FEW_ORIGINAL_SHARDS;
    }
    // one stream: pinned originals in, encode, pinned recovery rows out, one wait
    return guarded(err, [&]() -> rs_status {
        DeviceGuard dg(e->ctx->device);
        const hipStream_t s = e->st.get();
        const Geom g{e->row, uint32_t(e->row / 8)};
        auto *d_orig = static_cast<uint8_t *>(e->d_orig.get(e->N * e->row));
        auto *d_rec = static_cast<uint8_t *>(e->d_rec.get(e->M * e->row));
        uint8_t *h_rec = e->h_rec.get(e->M * e->row);
        check(hipMemcpyAsync(d_orig, e->h_orig.p, e->N * e->row, hipMemcpyHostToDevice, s));
        if (e->high) encode_high(e->ctx, e->ws, g, e->N, e->M, d_orig, d_rec, s);
        else encode_low(e->ctx, e->ws, g, e->N, e->M, d_orig, d_rec, s);
        check(hipMemcpyAsync(h_rec, d_rec, e->M * e->row, hipMemcpyDeviceToHost, s));
        check(hipStreamSynchronize(s));
        if (e->S != e->row) {  // tails: the reference's unpadded shards (shards.rs:62-74)
            e->h_tail.resize(e->M * e->S);
            for (uint64_t i = 0; i < e->M; ++i) extract_row(&e->h_tail[i * e->S], h_rec + i * e->row, e->S);
        }
        e->has_result = true;
        return set_err(err, RS_OK);
    });
}

const uint8_t *rs_encoder_recovery(rs_encoder *e, uint64_t index) {
    if (!e || !e->has_result || index >= e->M) return nullptr;
    return e->S == e->row ? e->h_rec.p + index * e->row : &e->h_tail[index * e->S];
}

void rs_encoder_result_drop(rs_encoder *e) {
    if (e) encoder_drop_result(e);
}
int rs_encoder_is_high_rate(const rs_encoder *e) { return e ? e->high : -1; }
void rs_encoder_free(rs_encoder *e) { delete e; }

rs_status rs_encoder_into_parts(rs_encoder *e, rs_context **ctx_out, rs_encoder_work **work_out) {
    if (!e) return RS_ERR_INVALID_ARGUMENT;
    auto *w = new rs_encoder_work;
    w->device = e->ctx->device;
    w->swap(*e);
    if (ctx_out) *ctx_out = e->ctx;
    if (work_out) *work_out = w;
    else delete w;
    delete e;
    return RS_OK;
}

void rs_encoder_work_free(rs_encoder_work *w) { delete w; }

// ---- decoder ----------------------------------------------------------------

rs_status rs_decoder_new(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S, rs_decoder **out,
                         rs_error *err) {
    return rs_decoder_new_with_work(ctx, rate, N, M, S, nullptr, out, err);
}

rs_status rs_decoder_new_with_work(rs_context *ctx, rs_rate rate, uint64_t N, uint64_t M, uint64_t S,
                                   rs_decoder_work *work, rs_decoder **out, rs_error *err) {
    std::unique_ptr<rs_decoder_work> w(work);  // consumed in every case
    if (!ctx || !out) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    *out = nullptr;
    auto *d = new rs_decoder;
    d->ctx = ctx;
    d->rate = rate;
    if (w) {
        if (w->device == ctx->device) w->swap(*d);
        else w->swap_host(*d);  // device buffers of another device: freed with w
    }
    const rs_status st = decoder_configure(d, N, M, S, err);
    if (st != RS_OK) {
        delete d;
        return st;
    }
    *out = d;
    return RS_OK;
}

rs_status rs_decoder_reset(rs_decoder *d, uint64_t N, uint64_t M, uint64_t S, rs_error *err) {
    if (!d) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    d->has_result = false;
    return decoder_configure(d, N, M, S, err);
}

// copy = false (one-shot rs_decode): check and mark the shard only; the caller
// copies the shards into the staging afterwards, in parallel
static rs_status dec_add(rs_decoder *d, bool orig, uint64_t index, const uint8_t *shard, uint64_t len, rs_error *err,
                         bool copy = true) {
    if (!d || (!shard && len)) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    decoder_drop_result(d);
    const uint64_t count = orig ? d->N : d->M;
    std::vector<uint8_t> &present = orig ? d->orig_present : d->rec_present;
    if (index >= count) {  // decoder_work.rs:70-74, 99-103
        set_err(err, orig ? RS_ERR_INVALID_ORIGINAL_SHARD_INDEX : RS_ERR_INVALID_RECOVERY_SHARD_INDEX);
        if (err) {
            (orig ? err->original_count : err->recovery_count) = count;
            err->index = index;
        }
        return rs_status(err ? err->code : RS_ERR_INVALID_ARGUMENT);
    }
    if (present[index]) {  // :75-76, :104-105
        set_err(err, orig ? RS_ERR_DUPLICATE_ORIGINAL_SHARD_INDEX : RS_ERR_DUPLICATE_RECOVERY_SHARD_INDEX);
        if (err) err->index = index;
        return orig ? RS_ERR_DUPLICATE_ORIGINAL_SHARD_INDEX : RS_ERR_DUPLICATE_RECOVERY_SHARD_INDEX;
    }
    if (len != d->S) {  // :77-81, :106-110
        set_err(err, RS_ERR_DIFFERENT_SHARD_SIZE);
        if (err) err->shard_bytes = d->S, err->got = len;
        return RS_ERR_DIFFERENT_SHARD_SIZE;
    }
    if (copy) insert_row((orig ? d->h_orig : d->h_rec).p + index * d->row, shard, d->S);
    present[index] = 1;
    ++(orig ? d->orig_received : d->rec_received);
    return set_err(err, RS_OK);
}

rs_status rs_decoder_add_original_shard(rs_decoder *d, uint64_t index, const uint8_t *shard, uint64_t len,
                                        rs_error *err) {
    return dec_add(d, true, index, shard, len, err);
}
rs_status rs_decoder_add_recovery_shard(rs_decoder *d, uint64_t index, const uint8_t *shard, uint64_t len,
                                        rs_error *err) {
    return dec_add(d, false, index, shard, len, err);
}

rs_status rs_decoder_decode(rs_decoder *d, rs_error *err) {
    if (!d) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    if (d->has_result) return set_err(err, RS_OK);
    if (d->orig_received + d->rec_received < d->N) {  // decoder_work.rs:125-130
        set_err(err, RS_ERR_NOT_ENOUGH_SHARDS);
        if (err)
            err->original_count = d->N, err->original_received_count = d->orig_received,
            err->recovery_received_count = d->rec_received;
        return RS_ERR_NOT_ENOUGH_SHARDS;
    }
    if (d->orig_received == d->N) {  // nothing to restore (decoder_work.rs:131-132)
        d->has_result = true;
        d->decoded = false;
        return set_err(err, RS_OK);
    }
    // one stream: only received rows in, decode, only restored rows out, one wait
    return guarded(err, [&]() -> rs_status {
        DeviceGuard dg(d->ctx->device);
        const hipStream_t s = d->st.get();
        const uint64_t row = d->row;
        const Geom g{row, uint32_t(row / 8)};
        auto *d_orig = static_cast<uint8_t *>(d->d_orig.get(d->N * row));
        auto *d_rec = static_cast<uint8_t *>(d->d_rec.get(d->M * row));
        auto *d_out = static_cast<uint8_t *>(d->d_out.get(d->N * row));
        uint8_t *h_out = d->h_out.get(d->N * row);
        // (absent rows of the device buffers and of h_out are scratch: copied runs may span them)
        copy_rows(d_orig, d->h_orig.p, row, row, d->orig_present.data(), 1, d->N, hipMemcpyHostToDevice, s, true);
        copy_rows(d_rec, d->h_rec.p, row, row, d->rec_present.data(), 1, d->M, hipMemcpyHostToDevice, s, true);
        decode_dev(d->ctx, d->ws, d->high, g, d->N, d->M, d_orig, d->orig_present.data(), d_rec,
                   d->rec_present.data(), d_out, s);
        copy_rows(h_out, d_out, row, row, d->orig_present.data(), 0, d->N, hipMemcpyDeviceToHost, s, true);
        check(hipStreamSynchronize(s));
        if (d->S != row) {  // tails: the reference's unpadded shards (shards.rs:62-74)
            d->h_tail.resize(d->N * d->S);
            for (uint64_t i = 0; i < d->N; ++i)
                if (!d->orig_present[i]) extract_row(&d->h_tail[i * d->S], h_out + i * row, d->S);
        }
        d->has_result = d->decoded = true;
        return set_err(err, RS_OK);
    });
}

const uint8_t *rs_decoder_restored_original(rs_decoder *d, uint64_t index) {
    if (!d || !d->has_result || !d->decoded || index >= d->N || d->orig_present[index]) return nullptr;
    return d->S == d->row ? d->h_out.p + index * d->row : &d->h_tail[index * d->S];
}

uint64_t rs_decoder_restored_count(const rs_decoder *d) {
    if (!d || !d->has_result || !d->decoded) return 0;
    return d->N - d->orig_received;
}

void rs_decoder_result_drop(rs_decoder *d) {
    if (d) decoder_drop_result(d);
}
int rs_decoder_is_high_rate(const rs_decoder *d) { return d ? d->high : -1; }
void rs_decoder_free(rs_decoder *d) { delete d; }

rs_status rs_decoder_into_parts(rs_decoder *d, rs_context **ctx_out, rs_decoder_work **work_out) {
    if (!d) return RS_ERR_INVALID_ARGUMENT;
    auto *w = new rs_decoder_work;
    w->device = d->ctx->device;
    w->swap(*d);
    if (ctx_out) *ctx_out = d->ctx;
    if (work_out) *work_out = w;
    else delete w;
    delete d;
    return RS_OK;
}

void rs_decoder_work_free(rs_decoder_work *w) { delete w; }

// ---- one-shot (lib.rs:251-353) -------------------------------------------------

}  // extern "C"
namespace {
// rows per CopyPool item: >= 64 KiB of copies each
uint64_t copy_rows_per_item(uint64_t S) { return std::max<uint64_t>(1, (uint64_t(64) << 10) / std::max<uint64_t>(1, S)); }
template <typename W>
W *pool_take(rs_context *ctx, std::vector<W *> &pool) {
    std::lock_guard<std::mutex> lock(ctx->pool_mu);
    if (pool.empty()) return nullptr;
    W *w = pool.back();
    pool.pop_back();
    return w;
}
template <typename W>
void pool_put(rs_context *ctx, std::vector<W *> &pool, W *w) {
    if (!w) return;
    {
        std::lock_guard<std::mutex> lock(ctx->pool_mu);
        if (pool.size() < rs_context::kOneShotPool) {
            pool.push_back(w);
            return;
        }
    }
    delete w;
}
}  // namespace
extern "C" {

rs_status rs_encode(rs_context *ctx, uint64_t N, uint64_t M, uint64_t S, const uint8_t *const *original,
                    uint64_t given, uint8_t *recovery_out, rs_error *err) {
    if (!ctx) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    if (use_high_rate(N, M) < 0) {  // lib.rs:264-269
        set_err(err, RS_ERR_UNSUPPORTED_SHARD_COUNT);
        if (err) err->original_count = N, err->recovery_count = M;
        return RS_ERR_UNSUPPORTED_SHARD_COUNT;
    }
    if (given == 0) {  // lib.rs:273-280
        set_err(err, RS_ERR_TOO_FEW_ORIGINAL_SHARDS);
        if (err) err->original_count = N, err->original_received_count = 0;
        return RS_ERR_TOO_FEW_ORIGINAL_SHARDS;
    }
    if (!original) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    (void)S;  // shard size is inferred from the first shard, as the reference does; S = its length
    rs_encoder *e = nullptr;
    rs_status st = rs_encoder_new_with_work(ctx, RS_RATE_DEFAULT, N, M, S, pool_take(ctx, ctx->enc_pool), &e, err);
    if (st != RS_OK) return st;
    CopyPool &cp = ctx->copies();
    const uint64_t per = copy_rows_per_item(S);
    // a null shard pointer takes the checked path (rs_encoder_add_original_shard's
    // RS_ERR_INVALID_ARGUMENT at that shard)
    bool all_shards = true;
    for (uint64_t i = 0; all_shards && S && i < std::min(given, N); ++i) all_shards = original[i] != nullptr;
    if (given <= N && all_shards) {
        // every shard is S bytes by this entry point's contract, so the per-shard checks
        // (encoder_work.rs:56-65) cannot fail: the shards go into the staging in parallel
        auto in = [&](uint64_t k) {
            for (uint64_t i = k * per; i < std::min(given, k * per + per); ++i)
                insert_row(e->h_orig.p + i * e->row, original[i], S);
        };
        const uint64_t items = (given + per - 1) / per;
        if (ctx->copyin_pool) cp.run(items, in);
        else
            for (uint64_t k = 0; k < items; ++k) in(k);
        e->received = given;
    } else {  // TooManyOriginalShards at shard N, after N were added (lib.rs:281-284); null shards
        for (uint64_t i = 0; i < given && st == RS_OK; ++i) st = rs_encoder_add_original_shard(e, original[i], S, err);
    }
    // (measured and dropped, profiles/r06j, r06l: the recovery rows straight into the
    // caller's pageable buffer, 149-154 against 117-120 us; the rows back in 2 / 4 / 8
    // pieces with the copy-out of each overlapping the next, 111-123 / 144-163 / 197-212
    // against 107-109 us -- every extra copy and event wait costs more than it hides)
    if (st == RS_OK) st = rs_encoder_encode(e, err);
    if (st == RS_OK && recovery_out)
        cp.run((M + per - 1) / per, [&](uint64_t k) {
            for (uint64_t i = k * per; i < std::min(M, k * per + per); ++i)
                std::memcpy(recovery_out + i * S, rs_encoder_recovery(e, i), S);
        });
    rs_encoder_work *w = nullptr;
    rs_encoder_into_parts(e, nullptr, &w);
    pool_put(ctx, ctx->enc_pool, w);
    return st;
}

rs_status rs_decode(rs_context *ctx, uint64_t N, uint64_t M, uint64_t S, const uint64_t *original_index,
                    const uint8_t *const *original, uint64_t original_given, const uint64_t *recovery_index,
                    const uint8_t *const *recovery, uint64_t recovery_given, uint8_t *restored_out,
                    uint8_t *restored_mask, rs_error *err) {
    if (!ctx) return set_err(err, RS_ERR_INVALID_ARGUMENT);
    if (restored_mask) std::memset(restored_mask, 0, N);
    if (use_high_rate(N, M) < 0) {  // lib.rs:310-315
        set_err(err, RS_ERR_UNSUPPORTED_SHARD_COUNT);
        if (err) err->original_count = N, err->recovery_count = M;
        return RS_ERR_UNSUPPORTED_SHARD_COUNT;
    }
    if (recovery_given == 0) {  // lib.rs:320-334
        if (original_given == N) return set_err(err, RS_OK);
        set_err(err, RS_ERR_NOT_ENOUGH_SHARDS);
        if (err) err->original_count = N, err->original_received_count = original_given;
        return RS_ERR_NOT_ENOUGH_SHARDS;
    }
    if ((original_given && (!original_index || !original)) || (recovery_given && (!recovery_index || !recovery)))
        return set_err(err, RS_ERR_INVALID_ARGUMENT);
    rs_decoder *d = nullptr;
    rs_status st = rs_decoder_new_with_work(ctx, RS_RATE_DEFAULT, N, M, S, pool_take(ctx, ctx->dec_pool), &d, err);
    if (st != RS_OK) return st;
    // shard lengths are S by construction of this C entry point; per-shard
    // lengths are checked by the Python / C++ front-ends that know them.  The
    // indices are checked in the reference's order (decoder_work.rs:62-117) first,
    // then the shards go into the staging in parallel (CopyPool)
    for (uint64_t i = 0; i < original_given && st == RS_OK; ++i)
        st = dec_add(d, true, original_index[i], original[i], S, err, false);
    for (uint64_t i = 0; i < recovery_given && st == RS_OK; ++i)
        st = dec_add(d, false, recovery_index[i], recovery[i], S, err, false);
    CopyPool &cp = ctx->copies();
    const uint64_t per = copy_rows_per_item(S), given = original_given + recovery_given;
    auto in = [&](uint64_t k) {
        for (uint64_t j = k * per; j < std::min(given, k * per + per); ++j) {
            const bool o = j < original_given;
            const uint64_t i = o ? j : j - original_given;
            insert_row((o ? d->h_orig : d->h_rec).p + (o ? original_index : recovery_index)[i] * d->row,
                       (o ? original : recovery)[i], S);
        }
    };
    if (st == RS_OK) {
        const uint64_t items = (given + per - 1) / per;
        if (ctx->copyin_pool) cp.run(items, in);
        else
            for (uint64_t k = 0; k < items; ++k) in(k);
    }
    if (st == RS_OK) st = rs_decoder_decode(d, err);
    if (st == RS_OK && d->decoded) {
        std::vector<uint64_t> miss;
        for (uint64_t i = 0; i < N; ++i)
            if (!d->orig_present[i]) {
                miss.push_back(i);
                if (restored_mask) restored_mask[i] = 1;
            }
        if (restored_out)
            cp.run((miss.size() + per - 1) / per, [&](uint64_t k) {
                for (uint64_t j = k * per; j < std::min<uint64_t>(miss.size(), k * per + per); ++j)
                    std::memcpy(restored_out + miss[j] * S, rs_decoder_restored_original(d, miss[j]), S);
            });
    }
    rs_decoder_work *w = nullptr;
    rs_decoder_into_parts(d, nullptr, &w);
    pool_put(ctx, ctx->dec_pool, w);
    return st;
}

// ---- Engine trait on device rows ------------------------------------------------

static rs_status engine_xform(rs_context *ctx, void *rows, uint64_t count, uint64_t len64, uint64_t pos,
                              uint64_t size, uint64_t trunc, uint64_t delta, void *stream, bool fft) {
    if (!ctx || !rows || size == 0 || (size & (size - 1)) || pos + size > count || trunc > size ||
        size > 65536 || delta + size > 65536 + 1)
        return RS_ERR_INVALID_ARGUMENT;
    return guarded(nullptr, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        const Geom g{len64 * 64, uint32_t(len64 * 8)};
        uint8_t *base = static_cast<uint8_t *>(rows) + pos * g.stride;
        auto s = static_cast<hipStream_t>(stream);
        const uint32_t n = uint32_t(size), L = ilog2(n);
        rs::PassArgs A = base_args(ctx, g, n);
        A.ifft_delta = A.fft_delta = uint32_t(delta);
        A.work_in = A.work_out = base;
        A.work_stride = g.stride;
        if (trunc < size) {
            // engine_naive.rs:43-105: each layer transforms only the butterfly groups that
            // start below truncated_size; rows at and past it keep what the upper layers
            // left there ("garbage", src/engine.rs:108-147).  One 1-bit pass per layer: the
            // sets of layer b (dist 2^b) whose group starts below trunc are a prefix.
            for (uint32_t i = 0; i < L; ++i) {
                const uint32_t b = fft ? L - 1 - i : i;
                const uint64_t groups = (trunc + (uint64_t(2) << b) - 1) >> (b + 1);
                if (groups) launch(1, fft ? rs::kFft : rs::kIfft, A, uint32_t(groups << b), b, s);
            }
            return RS_OK;
        }
        const Levels lv = levels(L, max_k_enc(g.packs));
        // in place: IFFT runs levels low -> high, FFT high -> low
        for (uint32_t i = 0; i < lv.m; ++i) {
            const uint32_t k = fft ? lv.m - 1 - i : i;
            run_level(A, lv, k, fft ? rs::kFft : rs::kIfft, n, s);
        }
        return RS_OK;
    });
}

rs_status rs_engine_fft(rs_context *ctx, void *d_rows, uint64_t shard_count, uint64_t shard_len_64, uint64_t pos,
                        uint64_t size, uint64_t truncated_size, uint64_t skew_delta, void *stream) {
    return engine_xform(ctx, d_rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, stream, true);
}
rs_status rs_engine_ifft(rs_context *ctx, void *d_rows, uint64_t shard_count, uint64_t shard_len_64, uint64_t pos,
                         uint64_t size, uint64_t truncated_size, uint64_t skew_delta, void *stream) {
    return engine_xform(ctx, d_rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, stream,
                        false);
}

rs_status rs_engine_mul(rs_context *ctx, void *d_rows, uint64_t block_count, uint16_t log_m, void *stream) {
    if (!ctx || (!d_rows && block_count)) return RS_ERR_INVALID_ARGUMENT;
    return guarded(nullptr, [&]() -> rs_status {
        DeviceGuard dg(ctx->device);
        check(rs::launch_mul(static_cast<uint8_t *>(d_rows), block_count, ctx->d_lut + size_t(log_m) * rs::kPermWords,
                             static_cast<hipStream_t>(stream)));
        return RS_OK;
    });
}

rs_status rs_engine_formal_derivative(rs_context *ctx, void *d_rows, uint64_t count, uint64_t len64, void *stream) {
    // utils.rs:99-104 slices work[i .. i + lowbit(i)], in range only for 2^k rows
    if (!ctx || (!d_rows && count) || (count & (count - 1))) return RS_ERR_INVALID_ARGUMENT;
    return guarded(nullptr, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        const uint64_t bytes = count * len64 * 64;
        auto s = static_cast<hipStream_t>(stream);
        StreamWs sw(ctx, s);
        auto *tmp = static_cast<uint8_t *>(sw.w.buf[0].get(bytes));
        check(hipMemcpyAsync(tmp, d_rows, bytes, hipMemcpyDeviceToDevice, s));
        check(rs::launch_formal_derivative(tmp, static_cast<uint8_t *>(d_rows), uint32_t(count), len64 * 64, s));
        return RS_OK;
    });
}

// ---- Engine trait over HOST shard arrays (the reference's ShardsRefMut) ----------

namespace {
// rows [pos, pos + size) of a host array -> device staging -> transform -> back
rs_status engine_xform_host(rs_context *ctx, uint8_t *rows, uint64_t count, uint64_t len64, uint64_t pos,
                            uint64_t size, uint64_t trunc, uint64_t delta, bool fft) {
    if (!ctx || !rows || !len64 || size == 0 || (size & (size - 1)) || pos + size > count || trunc > size ||
        size > 65536 || delta + size > 65536 + 1)
        return RS_ERR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lock(ctx->host_engine_mu);  // the staging buffer, for the whole round trip
    rs_status st = guarded(nullptr, [&]() -> rs_status {
        DeviceGuard dg(ctx->device);
        const uint64_t bytes = size * len64 * 64;
        void *d = ctx->host_engine_buf.get(bytes);
        check(hipMemcpy(d, rows + pos * len64 * 64, bytes, hipMemcpyHostToDevice));
        return RS_OK;
    });
    // the device transform on the null stream, between the two blocking copies
    if (st == RS_OK) st = engine_xform(ctx, ctx->host_engine_buf.p, size, len64, 0, size, trunc, delta, nullptr, fft);
    if (st != RS_OK) return st;
    return guarded(nullptr, [&]() -> rs_status {
        DeviceGuard dg(ctx->device);
        check(hipMemcpy(rows + pos * len64 * 64, ctx->host_engine_buf.p, size * len64 * 64, hipMemcpyDeviceToHost));
        return RS_OK;
    });
}
}  // namespace

rs_status rs_engine_fft_host(rs_context *ctx, uint8_t *rows, uint64_t shard_count, uint64_t shard_len_64,
                             uint64_t pos, uint64_t size, uint64_t truncated_size, uint64_t skew_delta) {
    return engine_xform_host(ctx, rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, true);
}
rs_status rs_engine_ifft_host(rs_context *ctx, uint8_t *rows, uint64_t shard_count, uint64_t shard_len_64,
                              uint64_t pos, uint64_t size, uint64_t truncated_size, uint64_t skew_delta) {
    return engine_xform_host(ctx, rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, false);
}
rs_status rs_engine_mul_host(rs_context *ctx, uint8_t *blocks, uint64_t block_count, uint16_t log_m) {
    if (!ctx || (!blocks && block_count)) return RS_ERR_INVALID_ARGUMENT;
    if (!block_count) return RS_OK;
    return guarded(nullptr, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->host_engine_mu);
        DeviceGuard dg(ctx->device);
        const uint64_t bytes = block_count * 64;
        void *d = ctx->host_engine_buf.get(bytes);
        check(hipMemcpy(d, blocks, bytes, hipMemcpyHostToDevice));
        check(rs::launch_mul(static_cast<uint8_t *>(d), block_count, ctx->d_lut + size_t(log_m) * rs::kPermWords,
                             nullptr));
        check(hipMemcpy(blocks, d, bytes, hipMemcpyDeviceToHost));
        return RS_OK;
    });
}

rs_status rs_release_stream_scratch(rs_context *ctx, void *stream) {
    if (!ctx) return RS_ERR_INVALID_ARGUMENT;
    return guarded(nullptr, [&]() -> rs_status {
        std::lock_guard<std::mutex> lock(ctx->mu);
        DeviceGuard dg(ctx->device);
        auto s = static_cast<hipStream_t>(stream);
        auto it = ctx->ws_by_stream.find(s);
        if (it == ctx->ws_by_stream.end()) return RS_OK;
        check(hipStreamSynchronize(s));
        ctx->ws_erase(s);
        return RS_OK;
    });
}

rs_status rs_profile_enable(rs_context *ctx, int enable) {
    if (!ctx) return RS_ERR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->prof = enable != 0;
    return RS_OK;
}

rs_status rs_mono_enable(rs_context *ctx, int enable) {
    if (!ctx) return RS_ERR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->mono = (enable & 3) != 0;
    ctx->mono_all = (enable & 3) == 2;
    ctx->split = !(enable & 4);
    // + 8: 4-element packs only; + 16: 2-element packs wherever the staged kernel runs
    ctx->e2_max_packs = (enable & 8) ? 0u : (enable & 16) ? 0xFFFFFFFFu : ctx->e2_default;
    ctx->e2_encode = !(enable & 8);
    // + 32: lane kernel on, + 64: off (neither: the context's default)
    ctx->lane = (enable & 32) ? true : (enable & 64) ? false : ctx->lane_default;
    ctx->lane_max_l = (enable & 32) ? 10 : ctx->lane_max_l_default;
    // + 128: half-split 2^12-row transforms on, + 256: off
    ctx->half = (enable & 128) ? true : (enable & 256) ? false : ctx->half_default;
    // + 2048: quad encode on, + 4096: off
    ctx->quad = (enable & 2048) ? true : (enable & 4096) ? false : ctx->quad_default;
    // + 512: multi-chunk kernel on, + 1024: off
    ctx->chunks = (enable & 512) ? true : (enable & 1024) ? false : ctx->chunks_default;
    // (neither bit: the context's defaults, RS_MI355X_CHUNKS=2's forced routing included)
    ctx->chunks_forced = (enable & 512) ? true : (enable & 1024) ? false : ctx->chunks_forced_default;
    return RS_OK;
}

rs_status rs_check_device(rs_context *ctx) {
    if (!ctx) return RS_ERR_INVALID_ARGUMENT;
    return guarded(nullptr, [&]() -> rs_status {
        DeviceGuard dg(ctx->device);
        check(hipDeviceSynchronize());
        check(hipGetLastError());
        return RS_OK;
    });
}

int rs_profile_collect(rs_context *ctx, float *ms, uint64_t *bytes, const char **names, int max) {
    if (!ctx) return -1;
    std::lock_guard<std::mutex> lock(ctx->mu);
    static thread_local std::vector<std::string> keep;
    keep.clear();
    int n = 0;
    for (auto &r : ctx->recs) {
        if (n < max) {
            float t = 0;
            if (hipEventSynchronize(r.b) == hipSuccess) (void)hipEventElapsedTime(&t, r.a, r.b);
            if (ms) ms[n] = t;
            if (bytes) bytes[n] = r.bytes;
            keep.push_back(r.name);
            ++n;
        }
        ctx->pool.push_back(r.a);
        ctx->pool.push_back(r.b);
    }
    if (names)
        for (int i = 0; i < n; ++i) names[i] = keep[i].c_str();
    ctx->recs.clear();
    return n;
}

void rs_engine_eval_poly(uint16_t *erasures, uint64_t truncated_size) { rs::eval_poly_host(erasures, truncated_size); }

const uint16_t *rs_table_exp(void) { return rs::tables().exp.data(); }
const uint16_t *rs_table_log(void) { return rs::tables().log.data(); }
const uint16_t *rs_table_skew(void) { return rs::tables().skew.data(); }
const uint16_t *rs_table_log_walsh(void) { return rs::tables().log_walsh.data(); }
const uint32_t *rs_table_perm_by_log(void) { return rs::tables().perm_by_log.data(); }
const uint32_t *rs_table_perm_by_skew(void) { return rs::tables().perm_by_skew.data(); }

}  // extern "C"
