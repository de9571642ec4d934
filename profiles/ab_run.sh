#!/bin/bash
# GPU box: quick parity check, the full -m gpu suite, then the -D variants (profiles/variants.py) on the
# single-GPU step and on the sharded protocol at N=1.  Usage (repo root): bash profiles/ab_run.sh OUTDIR [--no-tests]
set -e
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
if [ "$2" != "--no-tests" ]; then
    timeout -k 10 150 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -k "solves_small_golden or select_paths" \
        --timeout 120 --timeout-method thread > "$OUT/quick.log" 2>&1
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
    tail -2 "$OUT/tests.log"
fi
timeout -k 10 900 python -u profiles/variants.py bench --steps 6 --dist > "$OUT/variants.txt" 2>&1
cat "$OUT/variants.txt"
