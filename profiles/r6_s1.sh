#!/bin/bash
# Round 6, session 1: block-cyclic slices for the key-owner protocol (each exchange part one block of the global queue,
# claimed as soon as it has arrived): the sharded GPU parity suite, then the world-1 key-pass measurement (a rank's
# whole sharded device work on one GPU, streams overlapping) with its busy union
O=${1:-gpurun_out/r6s1}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 3 $O/dist.log; [ $rc -eq 0 ] || exit $rc
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_kp1 -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_kp1.json 2> $O/tr_kp1.err || exit 1
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --top 16 | tail -3
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --exclude 'rccl|k_mt_' | tail -1
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1.json 2> $O/kp1.err || exit 1
SB_FORCE_DIST=1 SB_DIST_KP1=1 SB_DIST_BC=0 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_nobc.json 2> $O/kp1_nobc.err || exit 1
python3 -c "
import json
for f in ('kp1', 'kp1_nobc'):
    d = json.load(open('$O/' + f + '.json'))
    print(f, d['value'], d['ms_per_step'])"
