#!/bin/bash
# Round 4: 30-bit sort prefix up to 2^21 kept keys — engine + realistic tests, C4 golden, C4 / C3 bench lines
O=${1:-gpurun_out/r4sm}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_realistic.py tests/test_gpu_custom.py "tests/test_gpu_big.py::test_realistic_c4_w1m_oracle_golden" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for cfg in c4 c3; do
    extra=""; [ $cfg = c4 ] && extra="--realistic"
    timeout -k 10 300 python3 bench.py $extra --no-cpu-baseline --steps 12 --warmup 2 > $O/${cfg}_$round.json 2> $O/${cfg}_$round.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/${cfg}_$round.json').read().strip().splitlines()[-1]); p=d['phases_ms']; print('$cfg', $round, round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'select', p['ms_select'])"
  done
done
