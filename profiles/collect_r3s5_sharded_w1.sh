#!/bin/bash
# round 3, session 5: rocprofv3 profile of the sharded step at world 1 (SB_FORCE_DIST=1 bench.py: the same
# process, no launcher): kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and TCC hit/miss passes, each its
# own run; summarised by profiles/summarize.py (the window delimited by k_expand<true>)
#   bash profiles/collect_r3s5_sharded_w1.sh OUT_DIR
set -e
OUT=${1:-gpurun_out/prof_sh1}
ARGS="--no-cpu-baseline --steps 6 --warmup 0"
export TMPDIR=/tmp SB_FORCE_DIST=1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
RX='k_expand|k_apply|k_emit|k_ds_|k_dest|k_part|k_os_|k_gather|k_rgather|k_recv'
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_write.json" 2> "$OUT/write.err"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_tcc" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_tcc.json" 2> "$OUT/tcc.err"
python3 profiles/summarize.py "$OUT" --steps 6 --out "$OUT/r3s5_profile_sharded_summary.json" > "$OUT/summarize.txt" 2>&1
tail -12 "$OUT/summarize.txt"
