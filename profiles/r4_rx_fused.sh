#!/bin/bash
# Round 4: C4's emission with the key range and first select digit fused in (default) against the separate passes
# (SB_RX_FUSED=0): realistic parity, the C4 W=1M golden, then bench lines and one kernel trace
O=${1:-gpurun_out/r4rxf}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_realistic.py "tests/test_gpu_big.py::test_realistic_c4_w1m_oracle_golden" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lib in default rxnf; do
    if [ $lib = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=splendor-rl-gym_amd/splendor_amd/variants/lib_$lib.so; fi
    timeout -k 10 300 python3 bench.py --realistic --no-cpu-baseline --steps 12 --warmup 2 > $O/c4_${lib}_$round.json 2> $O/c4_${lib}_$round.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c4_${lib}_$round.json').read().strip().splitlines()[-1]); p=d['phases_ms']; print('c4', '$lib', $round, round(d['value']/1e6,1), 'M/s', d['ms_per_step'], p)"
  done
done
unset SPLENDOR_BEAM_LIB
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --realistic --no-cpu-baseline --steps 6 --warmup 0 > $O/trace.json 2> $O/trace.err
