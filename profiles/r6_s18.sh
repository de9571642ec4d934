#!/bin/bash
# Round 6, session 18: SQ counters of the sharded step's two big kernels in the world-1 key-pass run (SB_DIST_KP1):
# k_keys_a (the key pass) and k_claim_goc (the claims) — what binds each (three passes, each its own run)
O=${1:-gpurun_out/r6s18}; mkdir -p $O
export TMPDIR=/tmp
export SB_FORCE_DIST=1 SB_DIST_KP1=1
ARGS="--gpus 1 --no-cpu-baseline --steps 6 --warmup 0"
pass() {   # name counters...
    local name=$1; shift
    timeout -k 10 -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex 'k_keys_a|k_claim_goc' --output-format csv -d $O/$name -o run -- \
        python3 bench.py $ARGS > $O/$name.json 2> $O/$name.err
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
pass sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA || exit 1
pass sq3 SQ_LEVEL_WAVES SQ_INSTS_FLAT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_IFETCH || exit 1
pass tcc FETCH_SIZE || exit 1
pass tccw WRITE_SIZE || exit 1
python3 profiles/sq_summary.py $O --kernel 'k_keys_a' > $O/sq_k_keys_a.txt; grep -E "share_|per_wave|waves" $O/sq_k_keys_a.txt | head -20
python3 profiles/sq_summary.py $O --kernel 'k_claim_goc' > $O/sq_k_claim_goc.txt; grep -E "share_|per_wave|waves" $O/sq_k_claim_goc.txt | head -20
