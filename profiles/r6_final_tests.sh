#!/bin/bash
# Round 6, final tree: the whole -m gpu suite and smoke, each under its own limit, stop at the first failure
O=${1:-gpurun_out/r6final6}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; exit $rc
