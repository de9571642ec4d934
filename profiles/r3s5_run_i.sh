#!/bin/bash
# round 3, session 5: stream-priority A/B (noise producers' side stream at low priority), three rounds, after
# the engine parity tests
O=${1:-gpurun_out/s5i}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_realistic.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
