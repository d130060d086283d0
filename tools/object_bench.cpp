// Object-API benchmark through the C ABI, in the reference benchmark's scope
// (benches/benchmarks.rs:97-139): per call, every original shard added with
// rs_encoder_add_original_shard then rs_encoder_encode; for the decoder at 1 %
// and 100 % original loss, the provided originals and recovery shards added,
// then rs_decoder_decode.  Host shards in, host shards out: this is the path a
// Rust ReedSolomonEncoder / ReedSolomonDecoder takes through the INTEGRATION.md
// shim, so the rate includes both copies over the host link.
//
// Also: a decode with 30 % of the originals lost at random indices (scattered rows),
// and the one-shot rs_encode / rs_decode (src/lib.rs:251-353), which build a fresh
// encoder / decoder per call.
//
// Usage: rs_object_bench N M S iters warmup  ->  one JSON object on stdout.
// The restored shards are compared with the originals after the timed calls.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rs_mi355x.h"

namespace {
double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
[[noreturn]] void die(const char *what, rs_status st) {
    std::fprintf(stderr, "%s failed: %d (%s)\n", what, int(st), rs_last_device_error());
    std::exit(1);
}
}  // namespace

int main(int argc, char **argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s N M S iters warmup\n", argv[0]);
        return 2;
    }
    const uint64_t N = std::strtoull(argv[1], nullptr, 10), M = std::strtoull(argv[2], nullptr, 10),
                   S = std::strtoull(argv[3], nullptr, 10);
    const int iters = std::atoi(argv[4]), warmup = std::atoi(argv[5]);
    rs_context *ctx = nullptr;
    rs_status st = rs_context_create(0, &ctx);
    if (st != RS_OK) die("rs_context_create", st);

    std::mt19937_64 gen(1234);
    std::vector<std::vector<uint8_t>> orig(N, std::vector<uint8_t>(S));
    for (auto &r : orig)
        for (auto &b : r) b = uint8_t(gen());

    rs_encoder *enc = nullptr;
    if ((st = rs_encoder_new(ctx, RS_RATE_DEFAULT, N, M, S, &enc, nullptr)) != RS_OK) die("rs_encoder_new", st);
    auto encode_once = [&]() {
        for (uint64_t i = 0; i < N; ++i)
            if ((st = rs_encoder_add_original_shard(enc, orig[i].data(), S, nullptr)) != RS_OK)
                die("rs_encoder_add_original_shard", st);
        if ((st = rs_encoder_encode(enc, nullptr)) != RS_OK) die("rs_encoder_encode", st);
    };
    for (int i = 0; i < warmup; ++i) encode_once();
    double t0 = now();
    for (int i = 0; i < iters; ++i) encode_once();
    const double t_enc = (now() - t0) / iters;
    std::vector<std::vector<uint8_t>> rec(M, std::vector<uint8_t>(S));
    for (uint64_t i = 0; i < M; ++i) std::memcpy(rec[i].data(), rs_encoder_recovery(enc, i), S);

    rs_decoder *dec = nullptr;
    if ((st = rs_decoder_new(ctx, RS_RATE_DEFAULT, N, M, S, &dec, nullptr)) != RS_OK) die("rs_decoder_new", st);
    double t_dec[2] = {0, 0};
    bool ok = true;
    const int pcts[2] = {1, 100};
    for (int k = 0; k < 2; ++k) {
        // benchmarks.rs:113-118: the last ceil(min(N, M) * pct / 100) originals are
        // lost; as many recovery shards, from index 0, are provided
        const uint64_t lost = ((N < M ? N : M) * pcts[k] + 99) / 100, have = N - lost;
        auto decode_once = [&]() {
            for (uint64_t i = 0; i < have; ++i)
                if ((st = rs_decoder_add_original_shard(dec, i, orig[i].data(), S, nullptr)) != RS_OK)
                    die("rs_decoder_add_original_shard", st);
            for (uint64_t i = 0; i < lost; ++i)
                if ((st = rs_decoder_add_recovery_shard(dec, i, rec[i].data(), S, nullptr)) != RS_OK)
                    die("rs_decoder_add_recovery_shard", st);
            if ((st = rs_decoder_decode(dec, nullptr)) != RS_OK) die("rs_decoder_decode", st);
        };
        for (int i = 0; i < warmup; ++i) decode_once();
        t0 = now();
        for (int i = 0; i < iters; ++i) decode_once();
        t_dec[k] = (now() - t0) / iters;
        for (uint64_t i = have; i < N; ++i) {
            const uint8_t *p = rs_decoder_restored_original(dec, i);
            ok = ok && p && std::memcmp(p, orig[i].data(), S) == 0;
        }
    }
    // scattered loss: 30 % of min(N, M) originals at random indices (every lost row its
    // own run of rows to copy), as many recovery shards from index 0
    const uint64_t lost_sc = ((N < M ? N : M) * 30 + 99) / 100;
    std::vector<uint8_t> gone(N, 0);
    {
        std::vector<uint64_t> idx(N);
        for (uint64_t i = 0; i < N; ++i) idx[i] = i;
        std::shuffle(idx.begin(), idx.end(), gen);
        for (uint64_t i = 0; i < lost_sc; ++i) gone[idx[i]] = 1;
    }
    auto decode_scattered = [&]() {
        for (uint64_t i = 0; i < N; ++i)
            if (!gone[i] && (st = rs_decoder_add_original_shard(dec, i, orig[i].data(), S, nullptr)) != RS_OK)
                die("rs_decoder_add_original_shard", st);
        for (uint64_t i = 0; i < lost_sc; ++i)
            if ((st = rs_decoder_add_recovery_shard(dec, i, rec[i].data(), S, nullptr)) != RS_OK)
                die("rs_decoder_add_recovery_shard", st);
        if ((st = rs_decoder_decode(dec, nullptr)) != RS_OK) die("rs_decoder_decode", st);
    };
    for (int i = 0; i < warmup; ++i) decode_scattered();
    t0 = now();
    for (int i = 0; i < iters; ++i) decode_scattered();
    const double t_sc = (now() - t0) / iters;
    for (uint64_t i = 0; i < N; ++i)
        if (gone[i]) {
            const uint8_t *p = rs_decoder_restored_original(dec, i);
            ok = ok && p && std::memcmp(p, orig[i].data(), S) == 0;
        }

    // one-shot rs_encode / rs_decode (lib.rs:251-353): a fresh encoder / decoder per call
    std::vector<const uint8_t *> optr(N), rptr(M);
    for (uint64_t i = 0; i < N; ++i) optr[i] = orig[i].data();
    for (uint64_t i = 0; i < M; ++i) rptr[i] = rec[i].data();
    std::vector<uint8_t> rec_out(M * S), rest_out(N * S);
    auto oneshot_enc = [&]() {
        if ((st = rs_encode(ctx, N, M, S, optr.data(), N, rec_out.data(), nullptr)) != RS_OK) die("rs_encode", st);
    };
    for (int i = 0; i < warmup; ++i) oneshot_enc();
    t0 = now();
    for (int i = 0; i < iters; ++i) oneshot_enc();
    const double t_1e = (now() - t0) / iters;
    for (uint64_t i = 0; i < M; ++i) ok = ok && std::memcmp(&rec_out[i * S], rec[i].data(), S) == 0;
    const uint64_t lost1 = ((N < M ? N : M) + 99) / 100, have1 = N - lost1;
    std::vector<uint64_t> oidx(have1), ridx(lost1);
    for (uint64_t i = 0; i < have1; ++i) oidx[i] = i;
    for (uint64_t i = 0; i < lost1; ++i) ridx[i] = i;
    auto oneshot_dec = [&]() {
        if ((st = rs_decode(ctx, N, M, S, oidx.data(), optr.data(), have1, ridx.data(), rptr.data(), lost1,
                            rest_out.data(), nullptr, nullptr)) != RS_OK)
            die("rs_decode", st);
    };
    for (int i = 0; i < warmup; ++i) oneshot_dec();
    t0 = now();
    for (int i = 0; i < iters; ++i) oneshot_dec();
    const double t_1d = (now() - t0) / iters;
    for (uint64_t i = have1; i < N; ++i) ok = ok && std::memcmp(&rest_out[i * S], orig[i].data(), S) == 0;

    const double bytes = double(N + M) * double(S), gib = 1024.0 * 1024.0 * 1024.0;
    std::printf(
        "{\"encode_GiBps\": %.3f, \"encode_us\": %.2f, \"decode_1pct_GiBps\": %.3f, \"decode_1pct_us\": %.2f, "
        "\"decode_100pct_GiBps\": %.3f, \"decode_100pct_us\": %.2f, \"decode_scattered30_GiBps\": %.3f, "
        "\"decode_scattered30_us\": %.2f, \"oneshot_encode_GiBps\": %.3f, \"oneshot_encode_us\": %.2f, "
        "\"oneshot_decode_1pct_GiBps\": %.3f, \"oneshot_decode_1pct_us\": %.2f, \"restored_ok\": %s, "
        "\"iters\": %d}\n",
        bytes / t_enc / gib, t_enc * 1e6, bytes / t_dec[0] / gib, t_dec[0] * 1e6, bytes / t_dec[1] / gib,
        t_dec[1] * 1e6, bytes / t_sc / gib, t_sc * 1e6, bytes / t_1e / gib, t_1e * 1e6, bytes / t_1d / gib,
        t_1d * 1e6, ok ? "true" : "false", iters);
    rs_decoder_free(dec);
    rs_encoder_free(enc);
    rs_context_destroy(ctx);
    return ok ? 0 : 1;
}
