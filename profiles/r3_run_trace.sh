#!/bin/bash
# round 3: serialised per-rank traces (device work and gloo staging copies under one lock) at world 2 and 8
O=${1:-gpurun_out/r3j}; mkdir -p $O
bash profiles/collect_r3_sharded.sh $O/w2 2 30 6 || exit $?
python3 profiles/sharded_table.py $O/w2 --world 2 --steps 6 --out $O/w2_table.json
bash profiles/collect_r3_sharded.sh $O/w8 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json
