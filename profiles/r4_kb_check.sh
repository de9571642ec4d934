#!/bin/bash
# Round 4: the key-owner record pack with batched loads — sharded parity, then world-8 serialised key-owner traces
O=${1:-gpurun_out/r4kb}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/key 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/key --world 8 --steps 5 --out $O/key_table.json | grep -v "^rank" | tail -19
python3 profiles/project_n8.py $O/key_table.json $O/key/bench_r0.json --single-ms 4.507 | grep -v "^{"
