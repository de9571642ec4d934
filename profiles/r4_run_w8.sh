#!/bin/bash
# C5 world-8 parity (one GPU, gloo) with the key pass, then serialised per-rank traces of the sharded step at
# world 8 (C5 shape: 4M per rank, the 5-step saturated window of the W=32M solve) and the phase table
O=${1:-gpurun_out/r4w8}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_big.py -x -v --timeout 500 --timeout-method thread \
    -k "world8" > $O/c5_world8.txt 2>&1 || { tail -20 $O/c5_world8.txt; exit 1; }
tail -3 $O/c5_world8.txt
bash profiles/collect_r3_sharded.sh $O/w8 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json
