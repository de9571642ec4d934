#!/bin/bash
# Round 4 diagnostics (timing only, wrong orders): the LSD sort passes with no look-back (SB_OS_DBG=1) and with
# unscattered writes (2) against the default, one kernel trace each — why the first pass takes ~85 us and the others ~50
O=${1:-gpurun_out/r4osd}; mkdir -p $O
export TMPDIR=/tmp
for v in default osdbg1 osdbg2; do
  if [ $v = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=splendor-rl-gym_amd/splendor_amd/variants/lib_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/$v.json 2> $O/$v.err || exit 1
done
