#!/bin/bash
# Round 5, the tree after the MT jump change: the whole -m gpu suite, smoke, the driver's C3 command, C4
O=${1:-gpurun_out/r5final5}; mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; python3 -c "import json; d=json.load(open('$O/bench_n1.json')); print('C3', round(d['value']/1e6,1), d['ms_per_step'], d.get('phases_ms'))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --realistic --steps 12 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
rc=$?; python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('C4', round(d['value']/1e6,1), d['ms_per_step'], d.get('phases_ms'))"; exit $rc
