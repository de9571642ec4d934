#!/bin/bash
# Round 5, session 4: sharded GPU tests after the new-key count moved into the claim pass; the serialised world-8
# trace of the default build; C4's SQ passes + the realistic gem/pool-hash table A/B (r5_c4_sq.sh)
O=${1:-gpurun_out/r5s4}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_big.py tests/test_gpu_realistic.py -x -v -k "w4m or c4 or realistic" --timeout 300 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -1 $O/big.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/t_base 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t_base --world 8 --steps 5 --out $O/t_base_table.json | tail -20
rm -rf $O/t_base/r*/
bash profiles/r5_c4_sq.sh $O/c4
