#!/bin/bash
# round 3, session 5: top-k parity (payload prefetch in the partition writes), per-kernel trace of the two
# first-partition variants, then their C3 A/B in two interleaved rounds
O=${1:-gpurun_out/s5c}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_custom.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r3s5_trace_variants.sh $O/trace || exit $?
for round in 1 2; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
