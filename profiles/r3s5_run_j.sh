#!/bin/bash
# round 3, session 5: the whole -m gpu suite (epoch-stamped sort look-back, batched answer-bit test), then the
# look-back epoch A/B (three interleaved rounds) with one kernel trace per variant
O=${1:-gpurun_out/s5j}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r3s5_trace_variants.sh $O/trace > $O/trace.txt 2>&1 || exit $?
grep -E "lib_|k_os_pass|fillBuffer|k_os_begin|k_tk_sortsetup|k_os_hist" $O/trace.txt
for round in 1 2 3; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
