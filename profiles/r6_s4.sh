#!/bin/bash
# Round 6, session 4: sbd_goal_table waits for its own copy again (the pipelined key pass had turned it into a wait for
# the whole key pass): sharded GPU parity, the world-1 key-pass measurement (trace + busy union, block-cyclic against
# contiguous, host time per call)
O=${1:-gpurun_out/r6s4}; mkdir -p $O
export TMPDIR=/tmp
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
grep hostprof $O/kp1_hostprof.err | head -12
python3 -c "
import json
for f in ('kp1_bc', 'kp1_nobc', 'kp1_hostprof'):
    d = json.load(open('$O/' + f + '.json'))
    print(f, d['value'], d['ms_per_step'])"
