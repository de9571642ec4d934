#!/bin/bash
# Round 6, session 25: k_apply_w without the move-space re-derivation (a check only) and without the own-claim reads
# under global-order claims — sharded GPU parity + W=4M / C5 world-8 goldens, the world-1 key-pass run against the
# SB_APPLY_CHECK=1 build (interleaved twice) and a kernel trace of each
O=${1:-gpurun_out/r6s25}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 2 $O/big.log; [ $rc -eq 0 ] || exit $rc
D=splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so
kp1() {   # name, lib
    SPLENDOR_BEAM_LIB=$2 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$1.json 2> $O/kp1_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$1.json')); print('kp1 $1', round(d['value']/1e6,1), d['ms_per_step'])"
}
kp1 new_1 $D && kp1 chk_1 ab/libsb_applychk.so && kp1 new_2 $D && kp1 chk_2 ab/libsb_applychk.so || exit 1
for v in new chk; do
    L=$D; [ $v = chk ] && L=ab/libsb_applychk.so
    SPLENDOR_BEAM_LIB=$L SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o run -- \
        python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_$v.json 2> $O/tr_$v.err || exit 1
    python3 - <<PY
import csv
for r in csv.DictReader(open('$O/tr_$v/run_kernel_stats.csv')):
    if 'k_apply_w' in r['Name']: print('$v k_apply_w avg', round(float(r['AverageNs']) / 1e3, 1), 'us max', round(float(r['MaxNs']) / 1e3, 1))
PY
    rm -f $O/tr_$v/run_kernel_trace.csv
done
