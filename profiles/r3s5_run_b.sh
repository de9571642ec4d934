#!/bin/bash
# round 3, session 5: sharded GPU parity (batched answer bits), then the per-kernel trace of the top-k variants
O=${1:-gpurun_out/s5b}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_dist.log 2>&1
rc=$?; tail -2 $O/tests_dist.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r3s5_trace_variants.sh $O/trace
