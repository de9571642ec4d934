#!/bin/bash
# round 3, session 5 end: the whole -m gpu suite, the look-back epoch A/B (two interleaved rounds), smoke, the
# driver's bench command, sharded N=1, C4, then the C3 kernel profile of the final build and its summary
O=${1:-gpurun_out/s5k}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
tail -1 $O/bench_n1.json | cut -c1-400
SB_FORCE_DIST=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 12 --warmup 2 > $O/bench_sharded_n1.json 2> $O/bench_sharded_n1.err || exit $?
tail -1 $O/bench_sharded_n1.json | cut -c1-300
timeout -k 10 300 python3 -u bench.py --realistic --steps 12 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
tail -1 $O/bench_c4.json | cut -c1-300
bash profiles/collect_r3.sh $O/prof || exit $?
python3 profiles/summarize.py $O/prof --steps 6 --out $O/r3s5_profile_summary.json > $O/summarize.txt 2>&1 || exit $?
tail -16 $O/summarize.txt
