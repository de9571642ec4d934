#!/bin/bash
# Round 5: where C4's k_rexpand2 spends its time.  Counter list, then SQ passes (<= 8 SQ_ each,
# one rocprofv3 run per pass), then the kernel trace of the same window (timing; counters are never mixed with it)
O=${1:-gpurun_out/r5c4sq}; mkdir -p $O
export TMPDIR=/tmp
ARGS="--realistic --no-cpu-baseline --steps 6 --warmup 0"
RX='k_rexpand2'
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
pass() {   # name counters...
    local name=$1; shift
    timeout -k 10 -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv -d $O/$name -o run -- \
        python3 bench.py $ARGS > $O/$name.json 2> $O/$name.err
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
pass sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA || exit 1
pass sq3 SQ_LEVEL_WAVES SQ_INSTS_FLAT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_IFETCH || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $ARGS \
    > $O/trace.json 2> $O/trace.err || exit 1
