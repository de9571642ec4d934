#!/bin/bash
# Round 6, session 6: the world-1 key-pass measurement with the per-part claims beside the key passes — A/B of the engine
# stream's priority (SB_DIST_PRIO) and the claim grid (SB_GOC_GRID), two interleaved rounds
O=${1:-gpurun_out/r6s6}; mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  for v in base prio grid1024 prio_grid1024 grid512; do
    unset SB_DIST_PRIO SB_GOC_GRID
    case $v in prio) export SB_DIST_PRIO=1;; grid1024) export SB_GOC_GRID=1024;; prio_grid1024) export SB_DIST_PRIO=1 SB_GOC_GRID=1024;; grid512) export SB_GOC_GRID=512;; esac
    SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 12 --warmup 2 > $O/kp1_${v}_$round.json 2> $O/kp1_${v}_$round.err || { tail -3 $O/kp1_${v}_$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/kp1_${v}_$round.json')); print('$v', $round, d['value'], d['ms_per_step'])"
  done
done
unset SB_DIST_PRIO SB_GOC_GRID
