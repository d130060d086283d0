"""Generate tests/golden/golden_cases.json from the reference's own test data.

Reads /root/reference/src/test_util.rs *as text* (the SHA-256 recovery hashes
at test_util.rs:575-850) and pairs each hash with the (rate, original_count,
recovery_count, shard_bytes, seed, decoder loss pattern) that the reference's
tests use for it.  The loss patterns are transcribed from the cited test
functions.  Nothing of the reference is executed.

Run:  python tests/golden/make_golden.py   (only in the build container; the
GPU box never reads /root/reference).
"""
import json
import os
import re
import sys

REF = "/root/reference/src/test_util.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_cases.json")


def parse(text):
    consts = dict(re.findall(r'pub\(crate\) const (\w+): &str\s*=\s*"([0-9a-f]{64})";', text))
    tables = {}
    for name in ("DEFAULT_TINY", "HIGH_TINY", "LOW_TINY"):
        body = re.search(name + r": &\[\(usize, usize, u8, &str\)\] = &\[(.*?)\n\];", text, re.S).group(1)
        rows = []
        for n, m, seed, h in re.findall(r'\((\d+),\s*(\d+),\s*(\d+),\s*("?[\w]+"?)\)', body):
            h = h.strip('"')
            rows.append((int(n), int(m), int(seed), consts.get(h, h)))
        tables[name] = rows
    return consts, tables


def R(a, b):
    return [[a, b]]  # half-open index range


def main():
    if not os.path.exists(REF):
        sys.exit("reference not mounted; golden_cases.json is committed")
    consts, tables = parse(open(REF).read())
    cases = []

    def add(name, src, rate, n, m, s, seed, h, orig, rec):
        cases.append(dict(name=name, source=src, rate=rate, original_count=n, recovery_count=m,
                          shard_bytes=s, seed=seed, recovery_sha256=h,
                          decoder_original=orig, decoder_recovery=rec))

    # roundtrips_tiny: original [recovery_count..original_count), recovery [0..min)
    for tname, rate, src in (("DEFAULT_TINY", "default", "src/rate/rate_default.rs:365-380"),
                             ("HIGH_TINY", "high", "src/rate/rate_high.rs:343-356"),
                             ("LOW_TINY", "low", "src/rate/rate_low.rs:343-356")):
        for n, m, seed, h in tables[tname]:
            add(f"{tname}_{n}_{m}", src, rate, n, m, 1024, seed, h,
                R(m, n) if m < n else [], R(0, min(n, m)))

    C = consts
    add("HIGH_all_originals_missing", "src/rate/rate_high.rs:327-338", "high", 3, 3, 1024, 133, C["EITHER_3_3"], [], R(0, 3))
    add("HIGH_no_originals_missing", "src/rate/rate_high.rs:340-343", "high", 3, 2, 1024, 132, C["HIGH_3_2"], R(0, 3), [])
    add("HIGH_3000_30000", "src/rate/rate_high.rs:361-374", "high", 3000, 30000, 64, 14, C["HIGH_3000_30000_14"], [], R(0, 3000))
    add("HIGH_32768_32768", "src/rate/rate_high.rs:376-389", "high", 32768, 32768, 64, 11, C["EITHER_32768_32768_11"], [], R(0, 32768))
    add("HIGH_60000_3000", "src/rate/rate_high.rs:391-404", "high", 60000, 3000, 64, 12, C["HIGH_60000_3000_12"], R(3000, 60000), R(0, 3000))
    add("HIGH_34000_2000_s8", "src/rate/rate_high.rs:406-418", "high", 34000, 2000, 8, 123, C["HIGH_34000_2000_123_8"], R(0, 32000), R(0, 2000))
    add("LOW_all_originals_missing", "src/rate/rate_low.rs:327-338", "low", 3, 3, 1024, 133, C["EITHER_3_3"], [], R(0, 3))
    add("LOW_no_originals_missing", "src/rate/rate_low.rs:340-343", "low", 2, 3, 1024, 123, C["LOW_2_3"], [[0, 2]], [])
    add("LOW_3000_60000", "src/rate/rate_low.rs:361-374", "low", 3000, 60000, 64, 13, C["LOW_3000_60000_13"], [], R(0, 3000))
    add("LOW_30000_3000", "src/rate/rate_low.rs:376-389", "low", 30000, 3000, 64, 15, C["LOW_30000_3000_15"], R(3000, 30000), R(0, 3000))
    add("LOW_32768_32768", "src/rate/rate_low.rs:391-404", "low", 32768, 32768, 64, 11, C["EITHER_32768_32768_11"], [], R(0, 32768))
    add("LOW_2000_34000_s8", "src/rate/rate_low.rs:406-418", "low", 2000, 34000, 8, 123, C["LOW_2000_34000_123_8"], R(0, 2000), R(0, 32000))
    add("lib_roundtrip", "src/lib.rs:367-379", "default", 2, 3, 1024, 123, C["LOW_2_3"], [], [[0, 2]])

    def pts(xs):
        return [[x, x + 1] for x in xs]

    # two-round sequences: (rate, explicit_reset, [round_a, round_b]); each round
    # = (n, m, s, hash, decoder_original, decoder_recovery, seed)
    two = [
        ("high_implicit", "src/rate/rate_high.rs:423-431", "high", False,
         [(3, 2, 1024, C["HIGH_3_2"], [1], [0, 1], 132), (3, 2, 1024, C["HIGH_3_2_232"], [0], [0, 1], 232)]),
        ("high_explicit", "src/rate/rate_high.rs:433-441", "high", True,
         [(3, 2, 1024, C["HIGH_3_2"], [1], [0, 1], 132), (5, 2, 1024, C["HIGH_5_2"], [0, 2, 4], [0, 1], 152)]),
        ("low_implicit", "src/rate/rate_low.rs:423-431", "low", False,
         [(2, 3, 1024, C["LOW_2_3"], [], [0, 2], 123), (2, 3, 1024, C["LOW_2_3_223"], [], [1, 2], 223)]),
        ("low_explicit", "src/rate/rate_low.rs:433-441", "low", True,
         [(2, 3, 1024, C["LOW_2_3"], [], [0, 2], 123), (2, 5, 1024, C["LOW_2_5"], [], [0, 4], 125)]),
        ("default_implicit", "src/rate/rate_default.rs:386-393", "default", False,
         [(2, 3, 1024, C["LOW_2_3"], [], [0, 2], 123), (2, 3, 1024, C["LOW_2_3_223"], [0], [1], 223)]),
        ("default_high_to_high", "src/rate/rate_default.rs:395-402", "default", True,
         [(3, 2, 1024, C["HIGH_3_2"], [1], [0, 1], 132), (5, 3, 1024, C["HIGH_5_3"], [1, 3], [0, 1, 2], 153)]),
        ("default_high_to_low", "src/rate/rate_default.rs:404-411", "default", True,
         [(3, 2, 1024, C["HIGH_3_2"], [1], [0, 1], 132), (2, 3, 1024, C["LOW_2_3"], [], [0, 2], 123)]),
        ("default_low_to_high", "src/rate/rate_default.rs:413-420", "default", True,
         [(2, 3, 1024, C["LOW_2_3"], [], [0, 1], 123), (3, 2, 1024, C["HIGH_3_2"], [1], [0, 1], 132)]),
        ("default_low_to_low", "src/rate/rate_default.rs:422-429", "default", True,
         [(2, 3, 1024, C["LOW_2_3"], [], [0, 2], 123), (3, 5, 1024, C["LOW_3_5"], [], [0, 2, 4], 135)]),
        ("reed_solomon_low_to_high", "src/reed_solomon.rs:247-273", "default", True,
         [(2, 3, 1024, C["LOW_2_3"], [], [0, 1], 123), (3, 2, 1024, C["HIGH_3_2"], [1], [0, 1], 132)]),
    ]
    rounds = []
    for name, src, rate, explicit, rr in two:
        rounds.append(dict(name=name, source=src, rate=rate, explicit_reset=explicit,
                           rounds=[dict(original_count=n, recovery_count=m, shard_bytes=s, recovery_sha256=h,
                                        decoder_original=pts(o), decoder_recovery=pts(r), seed=seed)
                                   for (n, m, s, h, o, r, seed) in rr]))

    json.dump(dict(generated_from="/root/reference/src/test_util.rs (hashes) + cited test functions (loss patterns)",
                   single=cases, two_rounds=rounds), open(OUT, "w"), indent=1)
    print(f"wrote {len(cases)} single cases, {len(rounds)} two-round sequences -> {OUT}")


if __name__ == "__main__":
    main()
