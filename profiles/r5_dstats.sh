#!/bin/bash
# Round 5: where the key-owner protocol's owner claims lose to the single GPU's fused pass.
#  1. claim outcomes per turn (SB_CLAIM_STATS variant: inserted / earlier-turn key / same-turn early-out / lost at
#     the atomicMin / displaced a holder, for own children and for received records), world 8 on one GPU, C5 shape,
#     round-4 claims (own children in the key pass, received records per part on arrival) against global-order
#     claims (SB_DIST_GOC=1: own children as records, one claim pass over all records in (source, part) order)
#  2. serialised per-rank kernel traces of the same two settings (collect_r3_sharded.sh) and their phase tables
O=${1:-gpurun_out/r5ds}; mkdir -p $O
LIB=$PWD/splendor-rl-gym_amd/splendor_amd/variants/lib_stats.so
stats() {   # tag goc
    local PORT=$((20000 + RANDOM % 20000)) pids=() rc=0
    for r in 0 1 2 3 4 5 6 7; do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=8 LOCAL_WORLD_SIZE=8 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        SB_DIST_BACKEND=gloo SB_VISITED_LOG2=29 SB_DIST_FLAGS=32 SB_DIST_GOC=$2 SPLENDOR_BEAM_LIB=$LIB \
        timeout -k 10 500 python3 bench.py --gpus 8 --no-cpu-baseline --steps 5 --warmup 0 > $O/$1_r$r.json 2> $O/$1_r$r.err &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait "$p" || rc=1; done
    grep -h dclaims $O/$1_r*.err | sort -k5,5n -k3,3n > $O/$1_dclaims.txt
    return $rc
}
stats goc0 0 || exit 1
stats goc1 1 || exit 1
for G in 0 1; do
    SB_DIST_GOC=$G bash profiles/collect_r3_sharded.sh $O/t_goc$G 8 29 5 || exit 1
    python3 profiles/sharded_table.py $O/t_goc$G --world 8 --steps 5 --out $O/t_goc${G}_table.json | tail -20
    rm -rf $O/t_goc$G/r*/   # the raw traces (the table keeps the phases)
done
