#!/bin/bash
# Round 5, session 21: (a) the grouped records' rows and entries in one pass (k_gkr_scatter, SB_GKR_FUSED=1) against
# the two scatters (lib_gkrsep); (b) a visited-set growth whose allocation loses a race with another rank on the GPU
# falls back to a smaller table or none (the C5 world-8 card-set golden OOMed that way in session r5final3).  Sharded
# suite, the C5 world-8 goldens, then the world-8 serialised tables of both builds
O=${1:-gpurun_out/r5s21}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "world8" --timeout 600 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -1 $O/big.log; [ $rc -eq 0 ] || exit $rc
for L in default gkrsep; do
    if [ $L = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$V/lib_$L.so; fi
    bash profiles/collect_r3_sharded.sh $O/kh_$L 8 29 5 || exit 1
    python3 profiles/sharded_table.py $O/kh_$L --world 8 --steps 5 --out $O/kh_${L}_table.json > $O/kh_${L}_table.txt
    python3 -c "import json; d=json.load(open('$O/kh_${L}_table.json')); k=d['robust_per_kernel_ms']; m=d['robust_mean_ms']; print('$L', 'rebalance', round(m['rebalance partition'],3), 'scatter', round(k.get('k_gkr_scatter',0)+k.get('k_part_scatter<9>',0)+k.get('k_part_scatter<10>',0),3), 'device', round(m['device total (engine stream)'],3))"
    rm -rf $O/kh_$L/r*/
done
