#!/bin/bash
# Kernel traces of the sharded step at world N on ONE GPU (round 3): one rocprofv3 process per rank (each
# runs python3 directly: no launcher under the profiler), gloo transport, SB_DIST_SERIALIZE=1 so every
# rank's backend calls run alone on the device (the trace's durations are one rank's own-GPU time).
#   bash profiles/collect_r3_sharded.sh OUT_DIR WORLD [VISITED_LOG2] [STEPS]   (STEPS <= the window: one engine)
#   python3 profiles/sharded_table.py OUT_DIR --world WORLD --steps 6
set -u
OUT=${1:-gpurun_out/prof_sh}
N=${2:-2}
VL=${3:-29}
STEPS=${4:-6}
export TMPDIR=/tmp
mkdir -p "$OUT"
PORT=$((20000 + RANDOM % 20000))
pids=()
for r in $(seq 0 $((N - 1))); do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    SB_DIST_BACKEND=gloo SB_DIST_SERIALIZE=1 SB_VISITED_LOG2=$VL SB_BENCH_PROGRESS=1 SB_DIST_FLAGS=32 \
    timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$OUT/r$r" -o run -- \
        python3 bench.py --gpus "$N" --no-cpu-baseline --steps "$STEPS" --warmup 0 > "$OUT/bench_r$r.json" 2> "$OUT/r$r.err" &
    pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
exit $rc
