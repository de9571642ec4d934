#!/bin/bash
# round 3, session 5: the whole -m gpu suite, the lost-mask clear A/B (two rounds), per-kernel trace of the
# default build, then the round-3 session-5 C3 profile (kernel trace + FETCH/WRITE/TCC passes) and its summary
O=${1:-gpurun_out/s5h}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
bash profiles/collect_r3.sh $O/prof || exit $?
python3 profiles/summarize.py $O/prof --steps 6 --out $O/r3s5_profile_summary.json > $O/summarize.txt 2>&1 || exit $?
tail -30 $O/summarize.txt
