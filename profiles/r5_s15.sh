#!/bin/bash
# Round 5, session 15: the emission's survivors as an LDS queue of (parent, move) entries (SB_EMIT_Q=768, default,
# in the survivor masks' LDS) against a search + 192-bit select per survivor (lib_emq0): the GPU suite without the
# C5 cases, then the C3 line, two interleaved rounds, with phases
O=${1:-gpurun_out/r5s15}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -k "not c5_" --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
    for L in default emq0; do
        LIB=$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so; [ $L != default ] && LIB=$V/lib_$L.so
        SPLENDOR_BEAM_LIB=$LIB timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 \
            > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err || exit 1
        python3 -c "import json,sys; d=json.load(open('$O/ab_${L}_$R.json')); print('$L', $R, round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
    done
done
