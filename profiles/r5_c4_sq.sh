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
# A/B: the realistic expansion's gem / pool hashes from the table (default) against folded per child
# (SB_RX2_NO_HTAB variant), two interleaved rounds of the C4 bench line
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
for R in 1 2; do
    for L in default rxnotab; do
        LIB=$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so; [ $L = rxnotab ] && LIB=$V/lib_rxnotab.so
        SPLENDOR_BEAM_LIB=$LIB timeout -k 10 300 python3 bench.py --realistic --no-cpu-baseline --steps 12 --warmup 2 \
            > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err || exit 1
        python3 -c "import json,sys; d=json.load(open('$O/ab_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
    done
done
