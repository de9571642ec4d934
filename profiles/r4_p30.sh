#!/bin/bash
# Round 4: the wave-per-run sort fix-up (k_fx_wave) — top-k tests and goldens with the default 40-bit prefix and
# with a 30-bit prefix (three LSD passes instead of four), then C3 / C4 bench lines of both (two rounds)
O=${1:-gpurun_out/r4p30}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py -x -v --timeout 300 --timeout-method thread > $O/tests40.log 2>&1
rc=$?; tail -1 $O/tests40.log; [ $rc -eq 0 ] || exit $rc
SPLENDOR_BEAM_LIB=splendor-rl-gym_amd/splendor_amd/variants/lib_p30.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_realistic.py -x -v --timeout 300 --timeout-method thread > $O/tests30.log 2>&1
rc=$?; tail -1 $O/tests30.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r4_sort_ab.sh $O default splendor-rl-gym_amd/splendor_amd/variants/lib_p30.so
