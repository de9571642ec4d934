#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box from the repo root), round 3.
# Pass 1: kernel trace + stats.  PMC passes each in their own run (MI355X_MICROARCH.md §rocprofv3 PMC
# slots: FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2, TCC_HIT_sum + TCC_MISS_sum 2).
#   profiles/collect_r3.sh OUT_DIR [bench args...]
set -e
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=${@:---no-cpu-baseline --steps 6 --warmup 0}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
RX='k_expand|k_count_lm|k_emit|k_tk_|k_os_|k_gather'
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_write.json" 2> "$OUT/write.err"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_tcc" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_tcc.json" 2> "$OUT/tcc.err"
