#!/bin/bash
# round 3: CLI GPU tests (incl. --gpus 2), then kernel traces of the sharded step: world 1 (plain), and
# serialised per-rank traces (device work and gloo staging copies under one lock) at world 2 and 8
O=${1:-gpurun_out/r3j}; mkdir -p $O/w1
timeout -k 10 600 python3 -u -m pytest tests/test_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_cli.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/tests_cli.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
SB_FORCE_DIST=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/w1/r0 -o run -- \
    python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/w1/bench.json 2> $O/w1/err.txt || exit $?
python3 profiles/sharded_table.py $O/w1 --world 1 --steps 6 --out $O/w1_table.json
bash profiles/collect_r3_sharded.sh $O/w2 2 30 6 || exit $?
python3 profiles/sharded_table.py $O/w2 --world 2 --steps 6 --out $O/w2_table.json
bash profiles/collect_r3_sharded.sh $O/w8 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json
