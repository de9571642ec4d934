#!/bin/bash
# Round 5, first GPU session: the sharded GPU tests (incl. the device-side RCCL completion double and the receive
# bound grown mid-turn), the W=4M sharded goldens (the claim diagnostics run separately: r5_dstats.sh)
O=${1:-gpurun_out/r5s1}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k w4m --timeout 400 --timeout-method thread > $O/w4m.log 2>&1
rc=$?; tail -2 $O/w4m.log; [ $rc -eq 0 ] || exit $rc
