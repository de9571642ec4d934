#!/bin/bash
# GPU box: profiles/round_end.sh, then the sel64 A/B (variants lib_new / lib_sub, two rounds, C3).
#   bash profiles/round_end_ab.sh OUTDIR
set -e
OUT=${1:-gpurun_out/round_end}
bash profiles/round_end.sh "$OUT"
for r in 1 2; do
    timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 >> "$OUT/variants.txt" 2>&1
done
cat "$OUT/variants.txt"
