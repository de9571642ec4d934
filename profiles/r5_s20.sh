#!/bin/bash
# Round 5, session 20: a claim that displaces a received record finds it by scanning its parent's
# records' tags — SB_MK_SCAN=8 tags per round trip (default) against one (lib_scan1): card-set parity, then the card-set
# world-8 serialised traces, two interleaved rounds
O=${1:-gpurun_out/r5s20}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
K="2-cfg14 or 3-cfg15 or 4-cfg16 or 2-cfg17 or 2-cfg18 or 3-cfg19 or 2-cfg20 or 3-cfg21 or 2-cfg22 or 3-cfg23 or 4-cfg24 or 2-cfg25 or 2-cfg26 or 3-cfg27 or 2-cfg29 or 4-cfg35 or 2-cfg36"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v -k "$K" --timeout 300 --timeout-method thread > $O/dist_mig.log 2>&1
rc=$?; tail -1 $O/dist_mig.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
  for L in default scan1; do
    if [ $L = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$V/lib_$L.so; fi
    bash profiles/collect_r4_mig.sh $O/mig_${L}_$R 8 29 5 288 || exit 1
    python3 profiles/sharded_table.py $O/mig_${L}_$R --world 8 --steps 5 --out $O/mig_${L}_${R}_table.json > $O/mig_${L}_${R}_table.txt
    python3 -c "import json; d=json.load(open('$O/mig_${L}_${R}_table.json')); k=d['robust_per_kernel_ms']; print('$L', $R, 'k_mkeys_a', round(k.get('k_mkeys_a',0),3), 'k_mig_claim', round(k.get('k_mig_claim',0),3), 'device', round(d['robust_mean_ms']['device total (engine stream)'],3))"
    rm -rf $O/mig_${L}_$R/r*/
  done
done
