#!/bin/bash
# round 3: sharded parity after the apply change (records carry their move), world-1 bench, world-8 trace
O=${1:-gpurun_out/r3i}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_claims.py "tests/test_gpu_big.py::test_sharded_w4m_oracle_golden" "tests/test_gpu_big.py::test_c5_sharded_world8_oracle_golden" -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -8
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
SB_FORCE_DIST=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 12 --warmup 2 > $O/bench_sharded_n1.json 2> $O/bench_sharded_n1.err || exit $?
tail -1 $O/bench_sharded_n1.json
bash profiles/collect_r3_sharded.sh $O/w8 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json
