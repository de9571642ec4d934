#!/bin/bash
# Round 5, session 3: sharded GPU tests + W=4M goldens after the position-free apply and the answers' lost bits folded
# into the bit packing (global-order claims); then serialised world-8 traces of the default build and of two key-pass
# grid variants (SB_KS_GRID_GOC 2048 / 4096)
O=${1:-gpurun_out/r5s3}; mkdir -p $O
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_big.py -x -v -k w4m --timeout 300 --timeout-method thread > $O/w4m.log 2>&1
rc=$?; tail -1 $O/w4m.log; [ $rc -eq 0 ] || exit $rc
for T in base ksg2048 ksg4096; do
    L=""; [ $T != base ] && L=$V/lib_$T.so
    SPLENDOR_BEAM_LIB=${L:-$PWD/splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so} \
        bash profiles/collect_r3_sharded.sh $O/t_$T 8 29 5 || exit 1
    python3 profiles/sharded_table.py $O/t_$T --world 8 --steps 5 --out $O/t_${T}_table.json | tail -4
    rm -rf $O/t_$T/r*/
done
