#!/bin/bash
# Round 4: the realistic GPU tests (goldens, stepwise vs the oracle, C4 at W=1M), then a C4 A/B of library
# builds (bench.py --realistic, two interleaved rounds): step time, phases, k_rexpand's roofline
#   bash profiles/r4_c4_ab.sh OUT_DIR LIB1 LIB2 ...   (LIB "default" = the in-tree build)
O=${1:-gpurun_out/r4c4ab}; shift; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_realistic.py "tests/test_gpu_big.py::test_realistic_c4_w1m_oracle_golden" \
    -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$lib; fi
    timeout -k 10 300 python3 bench.py --realistic --no-cpu-baseline --steps 12 --warmup 2 > $O/${name}_$round.json 2> $O/${name}_$round.err || { echo "$name failed"; tail -3 $O/${name}_$round.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${name}_$round.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', $round, round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms', d.get('phases_ms'), 'rexpand', r.get('launch_ms'), 'frac', r.get('frac'))"
  done
done
