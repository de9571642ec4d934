#!/bin/bash
# round 3: C5 world-8 parity (8 ranks on one GPU), then serialised per-rank traces at world 8
O=${1:-gpurun_out/r3f}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_big.py -k c5_sharded -x -v -s --timeout 900 --timeout-method thread > $O/tests_c5w8.log 2>&1
rc=$?
tail -3 $O/tests_c5w8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash profiles/collect_r3_sharded.sh $O/w8 8 29 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 6 --out $O/w8_table.json
