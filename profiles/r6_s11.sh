#!/bin/bash
# Round 6, session 11: where the sharded step's host time goes — cProfile of the world-1 key-pass run (SB_DIST_KP1)
O=${1:-gpurun_out/r6s11}; mkdir -p $O
export TMPDIR=/tmp
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 -m cProfile -o $O/kp1.prof bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1.json 2> $O/kp1.err || exit 1
python3 -c "
import pstats
p = pstats.Stats('$O/kp1.prof')
p.sort_stats('tottime').print_stats(45)
p.sort_stats('cumulative').print_stats(70)
" > $O/kp1_prof.txt 2>&1
python3 -c "import json; d=json.load(open('$O/kp1.json')); print('kp1', round(d['value']/1e6,1), d['ms_per_step'])"
