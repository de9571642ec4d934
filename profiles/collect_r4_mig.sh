#!/bin/bash
# Round 4: kernel traces of the sharded step with card-set ownership (flags bit 8) at world N on ONE GPU, as
# collect_r3_sharded.sh: one rocprofv3 process per rank, gloo transport, SB_DIST_SERIALIZE=1 (each rank's
# backend calls alone on the device), compact record buffers (flags bit 5: 8 ranks share the HBM).
#   bash profiles/collect_r4_mig.sh OUT_DIR WORLD [VISITED_LOG2] [STEPS] [FLAGS]
#   python3 profiles/sharded_table.py OUT_DIR --world WORLD --steps STEPS
set -u
OUT=${1:-gpurun_out/prof_mig}
N=${2:-8}
VL=${3:-28}
STEPS=${4:-5}
FL=${5:-288}
export TMPDIR=/tmp
mkdir -p "$OUT"
PORT=$((20000 + RANDOM % 20000))
pids=()
for r in $(seq 0 $((N - 1))); do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    SB_DIST_BACKEND=gloo SB_DIST_SERIALIZE=1 SB_VISITED_LOG2=$VL SB_BENCH_PROGRESS=1 SB_DIST_FLAGS=$FL \
    timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$OUT/r$r" -o run -- \
        python3 bench.py --gpus "$N" --no-cpu-baseline --steps "$STEPS" --warmup 0 > "$OUT/bench_r$r.json" 2> "$OUT/r$r.err" &
    pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
exit $rc
