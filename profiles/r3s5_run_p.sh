#!/bin/bash
# round 3, session 5: the whole -m gpu suite on the final tree (payload copy folded into the fix-up kernels,
# sort setup folded into the final partition's scan), smoke, the driver's bench command, then one kernel trace
O=${1:-gpurun_out/s5q}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
tail -1 $O/bench_n1.json | cut -c1-300
python3 -c "import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1]); print(d['phases_ms'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/bench_trace.json 2> $O/trace.err || exit $?
