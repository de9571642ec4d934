#!/bin/bash
# GPU box: kernel trace of the C3 bench per variant (profiles/variants.py build ...), one rocprofv3 run each.
# Usage: bash profiles/ab_trace.sh OUTDIR [bench args]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/abtrace}
shift || true
ARGS=${@:---no-cpu-baseline --steps 6 --warmup 1}
mkdir -p "$OUT"
for f in splendor-rl-gym_amd/splendor_amd/variants/lib_*.so; do
  v=$(basename $f .so)
  SPLENDOR_BEAM_LIB=$PWD/$f timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/$v" -o run -- python3 bench.py $ARGS > "$OUT/$v.json" 2> "$OUT/$v.err"
done
