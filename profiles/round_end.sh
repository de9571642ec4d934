#!/bin/bash
# GPU box, round end: the full -m gpu suite, smoke(), the driver's bench command, the sharded step at N=1
# and the C4 line.  Usage (repo root): bash profiles/round_end.sh OUTDIR
set -e
OUT=${1:-gpurun_out/round_end}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err"
tail -1 "$OUT/bench_n1.json"
SB_FORCE_DIST=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 12 --warmup 2 > "$OUT/bench_sharded_n1.json" 2> "$OUT/bench_sharded_n1.err"
tail -1 "$OUT/bench_sharded_n1.json"
timeout -k 10 300 python3 -u bench.py --realistic --steps 12 --warmup 2 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
tail -1 "$OUT/bench_c4.json"
