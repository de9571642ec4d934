#!/bin/bash
# Round 5, session 9: grouped kept records on the rebalance's wire (sbd_pack_kept_grouped /
# sbd_unpack_kept).  The sharded GPU tests (groups, the 20-byte form, 3-child split groups), the W=4M world-2 goldens,
# then the serialised world-8 trace of the default build and its N=8 projection
O=${1:-gpurun_out/r5s10}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m" --timeout 400 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -1 $O/big.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/t_gkr 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t_gkr --world 8 --steps 5 --out $O/t_gkr_table.json | tail -22
python3 profiles/project_n8.py $O/t_gkr_table.json $O/t_gkr/bench_r0.json | tail -5
rm -rf $O/t_gkr/r*/
