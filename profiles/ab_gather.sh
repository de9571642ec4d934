#!/bin/bash
# GPU box: k_gather_d variants (grid cap, next-descriptor prefetch), two interleaved rounds, C3 single GPU.
#   bash profiles/ab_gather.sh OUTDIR
set -e
OUT=${1:-gpurun_out/ab_gather}
mkdir -p "$OUT"
for r in 1 2; do
    timeout -k 10 600 python -u profiles/variants.py bench --steps 12 >> "$OUT/variants.txt" 2>&1
done
cat "$OUT/variants.txt"
