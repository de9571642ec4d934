#!/bin/bash
# Round 4: an 8-bit first LSD digit (38-bit prefix) against four 10-bit digits (40) — engine tests + C3/C5 goldens,
# realistic tests, then C3 / C4 bench lines (two rounds) and a C3 trace
O=${1:-gpurun_out/r4d0}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_realistic.py "tests/test_gpu_big.py::test_c5_w32m_single_gpu_oracle_golden" -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r4_sort_ab.sh $O default splendor-rl-gym_amd/splendor_amd/variants/lib_p40.so || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/trace.json 2> $O/trace.err
