#!/bin/bash
# Round 5, session 2: global-order claims with the ticketed claim pass (k_claim_goc, SB_GC_U rounds of 256 records per
# ticket): claim outcomes (SB_CLAIM_STATS variant) and serialised world-8 traces, C5 shape (as r5_dstats.sh); the
# default build (GC_U 8) and a GC_U 4 variant
O=${1:-gpurun_out/r5ds2}; mkdir -p $O
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
stats() {   # tag lib
    local PORT=$((20000 + RANDOM % 20000)) pids=() rc=0
    for r in 0 1 2 3 4 5 6 7; do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=8 LOCAL_WORLD_SIZE=8 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        SB_DIST_BACKEND=gloo SB_VISITED_LOG2=29 SB_DIST_FLAGS=32 SPLENDOR_BEAM_LIB=$2 \
        timeout -k 10 500 python3 bench.py --gpus 8 --no-cpu-baseline --steps 5 --warmup 0 > $O/$1_r$r.json 2> $O/$1_r$r.err &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait "$p" || rc=1; done
    grep -h dclaims $O/$1_r*.err | sort -k5,5n -k3,3n > $O/$1_dclaims.txt
    return $rc
}
stats gocT $V/lib_stats.so || exit 1
bash profiles/collect_r3_sharded.sh $O/t_gocT 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t_gocT --world 8 --steps 5 --out $O/t_gocT_table.json | tail -22
rm -rf $O/t_gocT/r*/
SPLENDOR_BEAM_LIB=$V/lib_gc4.so bash profiles/collect_r3_sharded.sh $O/t_gc4 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t_gc4 --world 8 --steps 5 --out $O/t_gc4_table.json | tail -22
rm -rf $O/t_gc4/r*/
