#!/bin/bash
# GPU box: top-k kernel times on random keys (profiles/sortbench.py) per variant under rocprofv3, then the
# top-k GPU tests and the C3 bench of the variants.  Usage: bash profiles/ab_sortdiag.sh OUTDIR
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/sortdiag}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -m gpu -x -q -k "topk or select or solves_small_golden" \
    --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
for f in splendor-rl-gym_amd/splendor_amd/variants/lib_*.so; do
  v=$(basename $f .so)
  SPLENDOR_BEAM_LIB=$PWD/$f timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 -u profiles/sortbench.py > "$OUT/$v.log" 2>&1
done
[ -n "$NOBENCH" ] || timeout -k 10 400 python3 -u profiles/variants.py bench --steps 12 > "$OUT/ab.txt" 2>&1
[ -n "$NOBENCH" ] || cat "$OUT/ab.txt"
