#!/bin/bash
# GPU box: emission A/B (variants lib_new / lib_old, two interleaved rounds, single + sharded N=1), then
# the SQ instruction-mix pass for both.  Usage (repo root): bash profiles/ab_emit.sh OUTDIR
set -e
OUT=${1:-gpurun_out/ab_emit}
mkdir -p "$OUT"
for r in 1 2; do
    timeout -k 10 600 python -u profiles/variants.py bench --steps 12 --dist >> "$OUT/variants.txt" 2>&1
done
cat "$OUT/variants.txt"
for v in new old; do
    export SPLENDOR_BEAM_LIB=$PWD/splendor-rl-gym_amd/splendor_amd/variants/lib_$v.so
    bash profiles/valu_emit.sh "$OUT/sq_$v"
done
