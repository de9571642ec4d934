#!/bin/bash
# Round 5, session 8: (a) C3's kernel trace (the select's kernels one by one); (b) the card-set
# protocol's world-8 serialised trace on this round's build (item 3: k_mkeys_a); (c) SQ passes of the world-2 key
# kernels, card-set (k_mkeys_a) and key-hash (k_keys_a, k_claim_goc), each rank alone on the device
O=${1:-gpurun_out/r5s8}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- \
    python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 > $O/c3.json 2> $O/c3.err || exit 1
cat $O/c3.json
bash profiles/collect_r4_mig.sh $O/mig8 8 29 5 288 || exit 1
python3 profiles/sharded_table.py $O/mig8 --world 8 --steps 5 --out $O/mig8_table.json | grep -E "expand|claims|device total"
rm -rf $O/mig8/r*/
N=2
sqpass() {   # name flags regex counters...
    local name=$1 fl=$2 rx=$3; shift 3
    local PORT=$((20000 + RANDOM % 20000)) pids=() rc=0
    mkdir -p $O/$name
    for r in 0 1; do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        SB_DIST_BACKEND=gloo SB_DIST_SERIALIZE=1 SB_BENCH_PROGRESS=1 SB_DIST_FLAGS=$fl \
        timeout -k 10 -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$rx" --output-format csv -d $O/$name/r$r -o run -- \
            python3 bench.py --gpus $N --no-cpu-baseline --steps 4 --warmup 0 > $O/$name/bench_r$r.json 2> $O/$name/r$r.err &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait "$p" || rc=$?; done
    return $rc
}
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
S2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
S3="SQ_LEVEL_WAVES SQ_INSTS_FLAT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_IFETCH"
for P in 1 2 3; do
    eval C=\$S$P
    sqpass mig_sq$P 256 'k_mkeys_a|k_expand' $C || exit 1
done
for P in 1 2 3; do
    eval C=\$S$P
    sqpass kh_sq$P 0 'k_keys_a|k_claim_goc|k_expand' $C || exit 1
done
python3 profiles/sq_summary.py $O --kernel 'k_mkeys_a|k_keys_a|k_claim_goc' > $O/sq_summary.txt; cat $O/sq_summary.txt | head -60
