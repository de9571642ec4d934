#!/bin/bash
# rocprofv3 collection for config C4 (bench.py --realistic), round 3: kernel trace + stats, then the PMC
# passes each in its own run (FETCH_SIZE: 3 TCC counters, WRITE_SIZE 2, TCC_HIT_sum + TCC_MISS_sum 2).
#   bash profiles/collect_r3_c4.sh OUT_DIR          (GPU box, repo root)
#   python3 profiles/summarize.py OUT_DIR --expand k_rexpand --steps 6 --out profiles/r3_c4_profile_summary.json
set -e
OUT=${1:-gpurun_out/prof_c4}
ARGS="--realistic --no-cpu-baseline --steps 6 --warmup 0"
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
RX='k_rexpand|k_count_lm|k_remit|k_tk_|k_os_|k_rgather'
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_write.json" 2> "$OUT/write.err"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_tcc" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_tcc.json" 2> "$OUT/tcc.err"
