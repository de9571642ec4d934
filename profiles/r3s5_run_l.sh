#!/bin/bash
# round 3, session 5: LSD digit width (8 / 10 bits) and pass occupancy (compiler's 155 VGPRs / capped at 128):
# engine parity on the default build and on the 10-bit variant, per-kernel traces, two interleaved C3 rounds
O=${1:-gpurun_out/s5l}; mkdir -p $O
V=splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_custom.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SPLENDOR_BEAM_LIB=$PWD/$V/lib_c_d10.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_custom.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_d10.log 2>&1
rc=$?; tail -2 $O/tests_d10.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r3s5_trace_variants.sh $O/trace > $O/trace.txt 2>&1 || exit $?
grep -E "lib_|k_os_pass|k_os_hist" $O/trace.txt
for round in 1 2; do
  timeout -k 10 600 python3 -u profiles/variants.py bench --steps 12 > $O/variants_$round.txt 2>&1 || exit $?
  cat $O/variants_$round.txt
done
