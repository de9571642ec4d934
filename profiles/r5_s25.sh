#!/bin/bash
# Round 5, session 25: the MT jump's correlation reads a poly word's 32 sequence words at once (SB_JR_WIDE=1)
# vs one LDS round trip per set bit (jr0): bit-exact MT tests, C3 A/B under the driver's command, C3 trace
O=${1:-gpurun_out/r5s25}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
V=splendor-rl-gym_amd/splendor_amd/variants
for R in 1 2 3; do
    for L in default jr0; do
        if [ $L = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$V/lib_$L.so; fi
        timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b_${L}_$R.json 2> $O/b_${L}_$R.err || exit 1
        python3 -c "import json; d=json.load(open('$O/b_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,1), d['ms_per_step'], round(d['value_engine_stream_end']/1e6,1))"
    done
done
unset SPLENDOR_BEAM_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- \
    python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 > $O/c3.json 2> $O/c3.err || exit 1
grep -h "k_mt" $O/c3/run_kernel_stats.csv | cut -c1-40,150-260
