#!/bin/bash
# A/B of the pass kernels' zero-twiddle top layer (RS_MONO_ZERO_TOP): variant zt0
# (tools/build_variant.sh zt0 "rs_kernels.hip" -DRS_MONO_ZERO_TOP=0) against the
# main build, alternating, per-launch times of config 4 / 5 encodes and decodes
# (tools/route_time.py; SHAPES overrides the shapes).  Output: gpurun_out/ab_zero_top/<variant>_<round>.jsonl
set -euo pipefail
source tools/ab_common.sh
OUT=gpurun_out/ab_zero_top
mkdir -p $OUT
for r in 1 2; do
  for v in ${VARIANT:-zt0} main; do
    use_lib $v
    timeout -k 10 240 python -u tools/route_time.py ${SHAPES:-8192:8192:65536 32768:32768:65536} --iters 5 > $OUT/${v}_$r.jsonl
  done
done
