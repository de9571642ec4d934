#!/bin/bash
# Round 4: the select tail in one workgroup (k_tk_tail) — engine, realistic and custom-heuristic tests + C4 golden,
# then C4 / C3 bench lines against SB_TK_TAIL_MAX=0 (two interleaved rounds)
O=${1:-gpurun_out/r4tail}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_realistic.py tests/test_gpu_custom.py "tests/test_gpu_big.py::test_realistic_c4_w1m_oracle_golden" "tests/test_gpu_big.py::test_c5_w32m_single_gpu_oracle_golden" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r4_sort_ab.sh $O default splendor-rl-gym_amd/splendor_amd/variants/lib_notail.so
