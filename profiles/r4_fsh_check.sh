#!/bin/bash
# Round 4: the fine fused select bins — engine goldens (single GPU), then the sort/select A/B bench lines
O=${1:-gpurun_out/r4fsh}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_custom.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r4_sort_ab.sh $O default splendor-rl-gym_amd/splendor_amd/variants/lib_fsh47.so splendor-rl-gym_amd/splendor_amd/variants/lib_lb16.so
