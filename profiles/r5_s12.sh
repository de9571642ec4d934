#!/bin/bash
# Round 5, session 12: (a) the group kernel skipping rounds with nothing kept (sharded GPU tests, world-8 trace of
# the default key-hash protocol); (b) VERDICT r4 item 3: k_mkeys_a's persistent grid held it at 4 waves per SIMD
# (1024 workgroups x 4 waves, SQ_WAVES 4096) where its LDS allows 7 and the single GPU's k_expand runs 8 — the
# card-set world-8 serialised trace at 1024 (default), 1536 and 1792 workgroups, card-set parity with the largest
O=${1:-gpurun_out/r5s12}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
SPLENDOR_BEAM_LIB=$V/lib_mkg1792.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v -k "2-cfg14 or 3-cfg15 or 4-cfg16 or 2-cfg17 or 2-cfg18 or 3-cfg19 or 2-cfg20 or 3-cfg21 or 2-cfg22 or 3-cfg23 or 4-cfg24 or 2-cfg25 or 2-cfg26 or 3-cfg27 or 2-cfg29 or 4-cfg33 or 2-cfg34" \
    --timeout 300 --timeout-method thread > $O/dist_mkg1792.log 2>&1
rc=$?; tail -1 $O/dist_mkg1792.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/t_gkr 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t_gkr --world 8 --steps 5 --out $O/t_gkr_table.json | grep -E "rebalance|receive|other|device total|per kernel"
python3 profiles/project_n8.py $O/t_gkr_table.json $O/t_gkr/bench_r0.json | grep "B=  400"
rm -rf $O/t_gkr/r*/
for L in default mkg1536 mkg1792; do
    if [ $L = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$V/lib_$L.so; fi
    bash profiles/collect_r4_mig.sh $O/mig_$L 8 29 5 288 || exit 1
    python3 profiles/sharded_table.py $O/mig_$L --world 8 --steps 5 --out $O/mig_${L}_table.json > $O/mig_${L}_table.txt
    python3 -c "import json; d=json.load(open('$O/mig_${L}_table.json')); k=d['robust_per_kernel_ms']; print('$L', 'k_mkeys_a', round(k.get('k_mkeys_a',0),3), 'device', round(d['robust_mean_ms']['device total (engine stream)'],3))"
    rm -rf $O/mig_$L/r*/
done
