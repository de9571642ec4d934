#!/bin/bash
# round 3: sharded-step traces at world 1 (torch-free serialisation not needed), 2 and 8 on one GPU
set -e
O=${1:-gpurun_out/r3c}; mkdir -p $O
mkdir -p $O/w1
# world 1: the plain sharded path (SB_FORCE_DIST), kernel trace of the timed window
SB_FORCE_DIST=1 SB_DIST_PHASES=0 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/w1/r0 -o run -- \
    python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/w1/bench.json 2> $O/w1/err.txt
python3 profiles/sharded_table.py $O/w1 --world 1 --steps 6 --out $O/w1_table.json
bash profiles/collect_r3_sharded.sh $O/w2 2 30
python3 profiles/sharded_table.py $O/w2 --world 2 --steps 6 --out $O/w2_table.json
bash profiles/collect_r3_sharded.sh $O/w8 8 29
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 6 --out $O/w8_table.json
