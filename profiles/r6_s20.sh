#!/bin/bash
# Round 6, session 20: the C5 world-8 goldens (W=32M over 8 ranks on one GPU) with 8 exchange parts per turn — 64
# blocks, the joint select at its 64-position limit with 8-bit digits — and with contiguous ranges (SB_DIST_BC=0)
O=${1:-gpurun_out/r6s20}; mkdir -p $O
export TMPDIR=/tmp
SB_DIST_PARTS=8 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "world8" --timeout 800 --timeout-method thread > $O/big_p8.log 2>&1
rc=$?; tail -n 2 $O/big_p8.log; [ $rc -eq 0 ] || exit $rc
SB_DIST_BC=0 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "world8" --timeout 800 --timeout-method thread > $O/big_nobc.log 2>&1
rc=$?; tail -n 2 $O/big_nobc.log; exit $rc
