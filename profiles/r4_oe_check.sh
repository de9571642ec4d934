#!/bin/bash
# Round 4: owner emission on the GPU — the sharded cases (tests/test_gpu_dist.py), then C5 at world 8 on one GPU
O=${1:-gpurun_out/r4oe}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -3 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest "tests/test_gpu_big.py::test_c5_sharded_world8_oracle_golden" -x -v --timeout 800 --timeout-method thread > $O/c5.log 2>&1
rc=$?; tail -3 $O/c5.log; exit $rc
