/* Sanitizer run of the CPU oracle (test infrastructure only): encode -> erase ->
 * decode round trips over both engines (naive restatement, AVX2 restatement),
 * every rate, tail sizes and multi-chunk shapes, built with
 * -fsanitize=address,undefined by `make -C oracle asan` (tests/test_oracle_golden.py
 * runs it).  Exit status 0 = every restored shard equals its original and no
 * sanitizer report. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_select_engine(int which);
int orc_encode(int rate, size_t N, size_t M, size_t S, const uint8_t *orig, uint8_t *rec);
int orc_decode(int rate, size_t N, size_t M, size_t S, const uint8_t *orig, const uint8_t *orig_present,
               const uint8_t *rec, const uint8_t *rec_present, uint8_t *out);
void orc_generate_original(size_t count, size_t S, uint8_t seed, uint8_t *out);

static int round_trip(int engine, int rate, size_t N, size_t M, size_t S, unsigned seed) {
    uint8_t *orig = malloc(N * S), *rec = malloc(M * S), *out = calloc(N, S);
    uint8_t *op = malloc(N), *rp = malloc(M);
    if (!orig || !rec || !out || !op || !rp) return 1;
    orc_generate_original(N, S, (uint8_t)seed, orig);
    if (orc_select_engine(engine) != 0) return 0; /* engine unavailable on this host */
    int err = orc_encode(rate, N, M, S, orig, rec);
    if (err) {
        fprintf(stderr, "encode error %d (rate %d %zu:%zu x %zu)\n", err, rate, N, M, S);
        return 1;
    }
    /* lose min(N, M) / 2 + 1 originals spread over the matrix, keep as many recovery shards */
    size_t lost = (N < M ? N : M) / 2 + 1;
    memset(op, 1, N);
    memset(rp, 0, M);
    for (size_t k = 0; k < lost; ++k) {
        op[(k * 7919u + seed) % N] = 0;
        rp[(k * 104729u + seed) % M] = 1;
    }
    size_t have_o = 0, have_r = 0;
    for (size_t i = 0; i < N; ++i) have_o += op[i];
    for (size_t i = 0; i < M; ++i) have_r += rp[i];
    int bad = 0;
    if (have_o + have_r >= N) {
        err = orc_decode(rate, N, M, S, orig, op, rec, rp, out);
        if (err) {
            fprintf(stderr, "decode error %d (rate %d %zu:%zu x %zu)\n", err, rate, N, M, S);
            bad = 1;
        }
        for (size_t i = 0; i < N && !bad; ++i)
            if (!op[i] && memcmp(out + i * S, orig + i * S, S)) {
                fprintf(stderr, "mismatch shard %zu (rate %d %zu:%zu x %zu)\n", i, rate, N, M, S);
                bad = 1;
            }
    }
    free(orig), free(rec), free(out), free(op), free(rp);
    orc_select_engine(0);
    return bad;
}

int main(void) {
    static const size_t shapes[][3] = {{1, 1, 64}, {3, 5, 64},   {5, 3, 2},     {2, 3, 30},    {100, 37, 130},
                                       {37, 100, 66}, {1000, 100, 128}, {100, 1000, 6}, {600, 200, 1000}};
    int fails = 0, runs = 0;
    for (int engine = 0; engine < 2; ++engine)
        for (int rate = 0; rate < 3; ++rate)
            for (size_t k = 0; k < sizeof shapes / sizeof shapes[0]; ++k) {
                fails += round_trip(engine, rate, shapes[k][0], shapes[k][1], shapes[k][2], (unsigned)(k + 3 * rate));
                ++runs;
            }
    printf("oracle sanitizer round trips: %d runs, %d failures\n", runs, fails);
    return fails != 0;
}
