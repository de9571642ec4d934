#!/bin/bash
# Round 6, session 12: exchange parts per turn with block-cyclic slices — the world-1 key-pass run (SB_DIST_KP1) at
# P = 2 / 4 / 8 parts, interleaved twice
O=${1:-gpurun_out/r6s12}; mkdir -p $O
export TMPDIR=/tmp
kp1() {   # name, parts
    SB_DIST_PARTS=$2 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$1.json 2> $O/kp1_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$1.json')); print('kp1 $1', round(d['value']/1e6,1), d['ms_per_step'])"
}
kp1 p4_1 4 && kp1 p8_1 8 && kp1 p2_1 2 && kp1 p4_2 4 && kp1 p8_2 8 && kp1 p2_2 2
