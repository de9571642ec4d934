#!/bin/bash
# round 3, session 5: the whole -m gpu suite on the default build, the driver's bench command, then the sharded
# step at N=1 with host time per call (profiles/r3s5_run_f.sh)
O=${1:-gpurun_out/s5g}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
tail -1 $O/bench_n1.json | cut -c1-700
bash profiles/r3s5_run_f.sh $O
