#!/bin/bash
# Round 5, session 11: the group kernel with batched destination loads (sharded GPU tests, the serialised world-8
# trace), then k_expand's SQ passes on C3 (one GPU) beside k_mkeys_a's (session 8) for VERDICT r4 item 3
O=${1:-gpurun_out/r5s11}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/t_gkr 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t_gkr --world 8 --steps 5 --out $O/t_gkr_table.json | grep -E "rebalance|receive|other|device total|k_gkr"
python3 profiles/project_n8.py $O/t_gkr_table.json $O/t_gkr/bench_r0.json | grep "B=  400"
rm -rf $O/t_gkr/r*/
ARGS="--no-cpu-baseline --steps 6 --warmup 0"
pass() {   # name counters...
    local name=$1; shift
    timeout -k 10 -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex 'k_expand' --output-format csv -d $O/$name -o run -- \
        python3 bench.py $ARGS > $O/$name.json 2> $O/$name.err
}
pass xp_sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
pass xp_sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA || exit 1
pass xp_sq3 SQ_LEVEL_WAVES SQ_INSTS_FLAT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_IFETCH || exit 1
python3 profiles/sq_summary.py $O --kernel 'k_expand' > $O/sq_k_expand.txt; grep -E "share_|per_wave" $O/sq_k_expand.txt
