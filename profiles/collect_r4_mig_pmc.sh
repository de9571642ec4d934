#!/bin/bash
# Round 4: the world > 1 key kernel's HBM traffic.  World 2 on ONE GPU, serialised
# (SB_DIST_SERIALIZE=1: each rank's backend calls alone on the device, so the device-wide TCC counters of a
# dispatch are that rank's), one rocprofv3 process per rank per pass: kernel trace, then FETCH_SIZE,
# WRITE_SIZE and TCC hit/miss, each its own run.  C5's shape: 4M states per rank, efficiency.
#   bash profiles/collect_r4_mig_pmc.sh OUT_DIR [FLAGS] [STEPS]   (FLAGS 257: card-set ownership + timing)
#   python3 profiles/pmc_sharded.py OUT_DIR --kernel k_mkeys_a --steps STEPS
set -u
OUT=${1:-gpurun_out/pmc_mig}
FL=${2:-257}
STEPS=${3:-4}
N=2
export TMPDIR=/tmp
mkdir -p "$OUT"
RX='k_mkeys_a|k_keys_a|k_mig_claim|k_own_claim_rec|k_apply_w|k_emit_w|k_mkeys_b|k_keys_b'
run_pass() {   # name, rocprofv3 args...
    local name=$1; shift
    local PORT=$((20000 + RANDOM % 20000)) pids=() rc=0
    for r in $(seq 0 $((N - 1))); do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        SB_DIST_BACKEND=gloo SB_DIST_SERIALIZE=1 SB_BENCH_PROGRESS=1 SB_DIST_FLAGS=$FL \
        timeout -k 10 600 rocprofv3 "$@" --output-format csv -d "$OUT/$name/r$r" -o run -- \
            python3 bench.py --gpus $N --no-cpu-baseline --steps "$STEPS" --warmup 0 > "$OUT/$name/bench_r$r.json" 2> "$OUT/$name/r$r.err" &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait "$p" || rc=$?; done
    return $rc
}
mkdir -p "$OUT/trace" "$OUT/fetch" "$OUT/write" "$OUT/tcc"
run_pass trace --kernel-trace || exit $?
run_pass fetch --pmc FETCH_SIZE --kernel-include-regex "$RX" || exit $?
run_pass write --pmc WRITE_SIZE --kernel-include-regex "$RX" || exit $?
run_pass tcc --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" || exit $?
