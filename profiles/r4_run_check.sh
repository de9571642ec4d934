#!/bin/bash
# round 4: the whole -m gpu suite, then the serialised world-8 sharded trace (pipelined key pass) and its table
O=${1:-gpurun_out/r4c}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -3 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/w8 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json | tail -16
