#!/bin/bash
# serialised per-rank traces of the sharded step at world 8 on one GPU (C5 shape: 4M per rank, the 5-step
# saturated window of the W=32M solve) and the phase table
O=${1:-gpurun_out/r4t}; mkdir -p $O
bash profiles/collect_r3_sharded.sh $O/w8 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json | tail -16
