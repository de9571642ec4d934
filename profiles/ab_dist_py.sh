#!/bin/bash
# GPU box: sharded step (SB_FORCE_DIST=1) with two versions of splendor_amd/dist.py (host protocol A/B).
# Usage: bash profiles/ab_dist_py.sh OUTDIR OLD.py NEW.py
set -e
OUT=$1; mkdir -p "$OUT"
cp splendor-rl-gym_amd/splendor_amd/dist.py "$OUT/dist_keep.py"
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then cp "$2" splendor-rl-gym_amd/splendor_amd/dist.py; else cp "$3" splendor-rl-gym_amd/splendor_amd/dist.py; fi
    SB_FORCE_DIST=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 12 --warmup 2 > "$OUT/b_$v$r.json" 2> "$OUT/b_$v$r.err"
    echo "$v $(python3 -c "import json,sys; d=json.loads(open('$OUT/b_$v$r.json').read().strip().splitlines()[-1]); print(d['ms_per_step'])")" >> "$OUT/ab.txt"
  done
done
cp "$OUT/dist_keep.py" splendor-rl-gym_amd/splendor_amd/dist.py
cat "$OUT/ab.txt"
