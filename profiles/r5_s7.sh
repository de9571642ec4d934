#!/bin/bash
# Round 5, session 7 (VERDICT r4 item 6, C3's select): three-pass LSD sorts of the kept keys' prefix — 11-bit digits
# over 33 or 32 bits, 12-bit digits over 36 — against the default four passes (8 + 3 x 10 = 38 bits); the fix-up orders
# any run of equal prefixes exactly.  Top-k tests with each variant first (exactness), then the C3 line, two
# interleaved rounds
O=${1:-gpurun_out/r5s7}; mkdir -p $O
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
for L in d11p33 d11p32; do
    SPLENDOR_BEAM_LIB=$V/lib_$L.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -x -q -k "topk" \
        --timeout 200 --timeout-method thread > $O/topk_$L.log 2>&1 || { tail -5 $O/topk_$L.log; exit 1; }
    tail -1 $O/topk_$L.log
done
for R in 1 2; do
    for L in default d11p33 d11p32; do
        LIB=$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so; [ $L != default ] && LIB=$V/lib_$L.so
        SPLENDOR_BEAM_LIB=$LIB SB_TOPK_STATS=$([ $R = 1 ] && echo 1 || echo "") timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 12 --warmup 2 \
            > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err || exit 1
        python3 -c "import json,sys; d=json.load(open('$O/ab_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
    done
done
