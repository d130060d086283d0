// GF(2^16) tables for the MI355X engine (host side, built once per process).
//
// Field: GF(2^16) with polynomial 0x1002D, elements in Cantor-basis coordinates
// (reference src/engine.rs:199-221, src/engine/tables.rs:184-324).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rs {

constexpr uint32_t kOrder = 65536;
constexpr uint32_t kModulus = 65535;

// Number of 32-bit words of one byte-permute multiply table (see PermTable).
constexpr int kPermWords = 20;
// Words of one table of the 2-element format (fill_perm2): a 32-bit word holds
// the low and the high byte of 2 elements, [lo0 lo1 hi0 hi1].
constexpr int kPerm2Words = 16;

struct GfTables {
    std::vector<uint16_t> exp;        // 65536, exp[65535] == exp[0]
    std::vector<uint16_t> log;        // 65536, log[0] == 65535
    std::vector<uint16_t> skew;       // 65536 (65535 used; last = 65535 pad)
    std::vector<uint16_t> log_walsh;  // 65536
    // lw_fold[(1<<u) - 1 + low] = sum_h log_walsh[h*2^u + low] mod 65535, u = 0..16
    std::vector<uint16_t> lw_fold;
    // Byte-permute multiply tables, kPermWords words per log_m (65536 entries).
    //   perm_by_log[log_m]   : x -> x * exp(log_m)       (Engine::mul semantics,
    //                           65535 == multiply by 1)
    //   perm_by_skew[idx]    : x -> x * exp(skew[idx]), or 0 when skew[idx] == 65535
    //                           (butterfly "no multiply" semantics,
    //                           engine_naive.rs:64-67 / 96-99)
    std::vector<uint32_t> perm_by_log;
    std::vector<uint32_t> perm_by_skew;
    // the same maps in the 2-element format (kPerm2Words words per entry)
    std::vector<uint32_t> perm2_by_log;
    std::vector<uint32_t> perm2_by_skew;

    uint16_t mul(uint16_t x, uint16_t log_m) const;
};

// Process-wide tables (thread-safe lazy init, like the reference's LazyLock).
const GfTables &tables();

uint16_t add_mod(uint16_t a, uint16_t b);
uint16_t sub_mod(uint16_t a, uint16_t b);

// Host eval_poly (reference src/engine/utils.rs:20-31), in place on 65536 values.
void eval_poly_host(uint16_t *erasures, size_t truncated);

}  // namespace rs
