#!/bin/bash
# Round 4: the card-set key pass at 7 waves per SIMD (four-wave blocks, compact LDS; default) and 8 (eight-wave
# blocks, SB_MK_NT 512): sharded parity first, then world-8 serialised traces with owner emission (flags 800)
O=${1:-gpurun_out/r4mko}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
for v in default mk512; do
  if [ $v = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=splendor-rl-gym_amd/splendor_amd/variants/lib_$v.so; fi
  bash profiles/collect_r4_mig.sh $O/$v 8 29 5 800 || exit $?
  python3 profiles/sharded_table.py $O/$v --world 8 --steps 5 --out $O/${v}_table.json | grep -E "expand|owner claims|device total"
done
