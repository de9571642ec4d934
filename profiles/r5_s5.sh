#!/bin/bash
# Round 5, session 5: the realistic expansion software-pipelined (SB_RX2_PIPE) — realistic tests and C4 at W=1M, then
# an A/B on the C4 bench line: default (pipelined, 5 waves) / not pipelined / pipelined at 4 waves, two interleaved rounds
O=${1:-gpurun_out/r5s5}; mkdir -p $O
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_realistic.py tests/test_gpu_big.py tests/test_gpu_growth.py -x -v -k "realistic or c4 or growth" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
    for L in default rxnopipe rxpipe4; do
        LIB=$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so; [ $L != default ] && LIB=$V/lib_$L.so
        SPLENDOR_BEAM_LIB=$LIB timeout -k 10 300 python3 bench.py --realistic --no-cpu-baseline --steps 12 --warmup 2 \
            > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err || exit 1
        python3 -c "import json,sys; d=json.load(open('$O/ab_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
    done
done
