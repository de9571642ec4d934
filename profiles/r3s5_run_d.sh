#!/bin/bash
# round 3, session 5: the whole -m gpu suite on the default build (payload prefetch, staged partition, fused
# survivor count + tile sums, coalesced scan), per-kernel trace of the variants, then their C3 A/B twice
O=${1:-gpurun_out/s5e}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r3s5_trace_variants.sh $O/trace || exit $?
for round in 1 2; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
