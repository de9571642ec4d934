#!/bin/bash
# Round 5, session 14: the key passes' children as an LDS queue of (parent, move) entries built lane-per-parent
# (SB_KS_Q=1024, default) instead of a binary search over the starts and a 192-bit select per child (lib_ksq0):
# sharded parity, then the world-8 serialised traces of both protocols, two interleaved rounds
O=${1:-gpurun_out/r5s14}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m" --timeout 400 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -1 $O/big.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
  for L in default ksq0; do
    if [ $L = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$V/lib_$L.so; fi
    bash profiles/collect_r3_sharded.sh $O/kh_${L}_$R 8 29 5 || exit 1
    python3 profiles/sharded_table.py $O/kh_${L}_$R --world 8 --steps 5 --out $O/kh_${L}_${R}_table.json > $O/kh_${L}_${R}_table.txt
    python3 -c "import json; d=json.load(open('$O/kh_${L}_${R}_table.json')); k=d['robust_per_kernel_ms']; print('kh $L', $R, 'k_keys_a', round(k.get('k_keys_a',0),3), 'device', round(d['robust_mean_ms']['device total (engine stream)'],3))"
    [ $R = 1 ] && [ $L = default ] && cp $O/kh_${L}_$R/bench_r0.json $O/kh_default_bench_r0.json
    rm -rf $O/kh_${L}_$R/r*/
  done
done
python3 profiles/project_n8.py $O/kh_default_1_table.json $O/kh_default_bench_r0.json | grep "B=  400"
for L in default ksq0; do
    if [ $L = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$V/lib_$L.so; fi
    bash profiles/collect_r4_mig.sh $O/mig_$L 8 29 5 288 || exit 1
    python3 profiles/sharded_table.py $O/mig_$L --world 8 --steps 5 --out $O/mig_${L}_table.json > $O/mig_${L}_table.txt
    python3 -c "import json; d=json.load(open('$O/mig_${L}_table.json')); k=d['robust_per_kernel_ms']; print('mig $L', 'k_mkeys_a', round(k.get('k_mkeys_a',0),3), 'device', round(d['robust_mean_ms']['device total (engine stream)'],3))"
    rm -rf $O/mig_$L/r*/
done
