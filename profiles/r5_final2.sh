#!/bin/bash
# Round 5, last build: the whole -m gpu suite, smoke, the driver's default bench line (N=1, with cpu_baseline), then
# the C3 kernel trace + PMC passes (collect_r3.sh) summarised — every step under its own time limit, stop at the first
# failure
O=${1:-gpurun_out/r5final2}; mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; cat $O/bench_n1.json; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3.sh $O/prof || exit $?
python3 profiles/summarize.py $O/prof --steps 6 --out $O/prof/r5_final2_profile_summary.json | tail -12
