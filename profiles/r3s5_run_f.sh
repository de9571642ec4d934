#!/bin/bash
# round 3, session 5: the sharded step at N=1 — host time inside every backend / collective call (which calls
# wait), then the plain bench line
O=${1:-gpurun_out/s5f}; mkdir -p $O
SB_FORCE_DIST=1 SB_DIST_HOSTPROF=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 12 --warmup 2 > $O/sharded_hostprof.json 2> $O/sharded_hostprof.err || exit $?
grep hostprof $O/sharded_hostprof.err | head -40
SB_FORCE_DIST=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 12 --warmup 2 > $O/sharded_n1.json 2> $O/sharded_n1.err || exit $?
tail -1 $O/sharded_n1.json
