#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats.  Passes 2/3: PMC FETCH_SIZE and WRITE_SIZE in their own runs
# (TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2 — MI355X_MICROARCH.md §rocprofv3 PMC slots).
set -e
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_expand|k_count_lm|k_emit|k_tk_|k_os_|k_gather' \
    --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_expand|k_count_lm|k_emit|k_tk_|k_os_|k_gather' \
    --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > "$OUT/bench_write.json" 2> "$OUT/write.err"
