#!/bin/bash
# Round 4: top-k tests + goldens after the LDS-staged tile scan, a C3 bench line and a kernel trace
O=${1:-gpurun_out/r4scan}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,1), 'M/s', d['ms_per_step'], d['phases_ms'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/trace.json 2> $O/trace.err
