#!/bin/bash
# Round 4 end, last build: the whole -m gpu suite, smoke and the driver's default bench line
O=${1:-gpurun_out/r4final6}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err
