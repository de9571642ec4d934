#!/bin/bash
# Round 5, session 16: the select histograms' LDS sub-histograms per 1024-thread block — 4 (default),
# 8, 16 — against the crowding of C3's scores (the prepass over all keys runs at 3.6-3.9 TB/s): top-k tests per variant,
# then the C3 line, two interleaved rounds, with phases and a kernel trace of each variant
O=${1:-gpurun_out/r5s16}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
for L in nh8 nh16; do
    SPLENDOR_BEAM_LIB=$V/lib_$L.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -x -q -k "topk" \
        --timeout 200 --timeout-method thread > $O/topk_$L.log 2>&1 || { tail -5 $O/topk_$L.log; exit 1; }
    tail -1 $O/topk_$L.log
done
for R in 1 2; do
    for L in default nh8 nh16; do
        LIB=$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so; [ $L != default ] && LIB=$V/lib_$L.so
        SPLENDOR_BEAM_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 12 --warmup 2 \
            > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err || exit 1
        python3 -c "import json,sys; d=json.load(open('$O/ab_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
    done
done
for L in default nh8; do
    LIB=$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so; [ $L != default ] && LIB=$V/lib_$L.so
    SPLENDOR_BEAM_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$L -o run -- \
        python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/tr_$L.json 2> $O/tr_$L.err || exit 1
    grep -E "k_tk_hist|k_tk_stage" $O/tr_$L/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
done
