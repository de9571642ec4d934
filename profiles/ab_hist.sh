#!/bin/bash
# GPU box: the -m gpu suite on the default build, then the histogram-flush and gather variants
# (profiles/variants.py), two interleaved rounds on C3.  Usage (repo root): bash profiles/ab_hist.sh OUTDIR
set -e
OUT=${1:-gpurun_out/ab_hist}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -2 "$OUT/tests.log"
for r in 1 2; do
    timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 >> "$OUT/variants.txt" 2>&1
done
cat "$OUT/variants.txt"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_exact.json" 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --lookahead-edges > "$OUT/bench_edges.json" 2>&1
tail -1 "$OUT/bench_exact.json" | cut -c1-400
tail -1 "$OUT/bench_edges.json" | cut -c1-400
