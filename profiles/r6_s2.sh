#!/bin/bash
# Round 6, session 2: records packed on the engine stream right behind each part's key pass (claims read the own records
# from the send buffer), host metadata over shared memory: sharded GPU parity, the world-1 key-pass measurement (trace +
# busy union, block-cyclic against contiguous), host time per call (SB_DIST_HOSTPROF)
O=${1:-gpurun_out/r6s2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 profiles/probe_cai.py > $O/cai.txt 2>&1; tail -n 2 $O/cai.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 3 $O/dist.log; [ $rc -eq 0 ] || exit $rc
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_kp1 -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_kp1.json 2> $O/tr_kp1.err || exit 1
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --top 16 | tail -3
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --exclude 'rccl|k_mt_' | tail -1
for v in bc nobc; do
  if [ $v = nobc ]; then export SB_DIST_BC=0; fi
  SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$v.json 2> $O/kp1_$v.err || exit 1
done
unset SB_DIST_BC
SB_FORCE_DIST=1 SB_DIST_KP1=1 SB_DIST_HOSTPROF=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 6 --warmup 2 > $O/kp1_hostprof.json 2> $O/kp1_hostprof.err || exit 1
grep hostprof $O/kp1_hostprof.err | head -40
python3 -c "
import json
for f in ('kp1_bc', 'kp1_nobc', 'kp1_hostprof'):
    d = json.load(open('$O/' + f + '.json'))
    print(f, d['value'], d['ms_per_step'])"
