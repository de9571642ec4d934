#!/bin/bash
# Round 6, session 15: part 0's blocks of the next beam smaller than the others' (SB_DIST_P0), so the claims, which wait
# for part 0's key pass, start sooner — the sharded GPU suite with SB_DIST_P0=0.5, then the world-1 key-pass run at
# P0 = 1 / 0.5 / 0.3, interleaved twice (the key-pass timing read moved after the rebalance)
O=${1:-gpurun_out/r6s15}; mkdir -p $O
export TMPDIR=/tmp
SB_DIST_P0=0.5 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
kp1() {   # name, p0
    SB_DIST_P0=$2 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$1.json 2> $O/kp1_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$1.json')); print('kp1 $1', round(d['value']/1e6,1), d['ms_per_step'])"
}
kp1 p10_1 1.0 && kp1 p05_1 0.5 && kp1 p03_1 0.3 && kp1 p10_2 1.0 && kp1 p05_2 0.5 && kp1 p03_2 0.3
