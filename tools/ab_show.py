"""Print the bench lines an A/B run (tools/ab_stream.sh) left under gpurun_out/<tag>/."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/c*.json") + glob.glob(f"gpurun_out/{sys.argv[1]}/*/c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    dec = {k: v for k, v in d.get("decode_GiBps", {}).items() if k in ("1pct", "100pct")}
    print(f, d["value"], "ms", d["ms_per_step"], "dec", dec, "enc_only", d.get("encode_only"))
    print("   ", {k: round(v["avg_us"], 1) for k, v in r.get("kernels", {}).items()})
