#!/bin/bash
# Round 5, session 22: (a) k_dest's tile histogram aggregated per wave and destination (SB_DEST_AGG=1) against an
# LDS atomic per kept key (lib_dagg0); (b) the key pass in 8 exchange parts instead of 4 (SB_DIST_PARTS=8: the last
# part's transfer, which the claims wait for, halves).  Sharded suite, then world-8 serialised tables
O=${1:-gpurun_out/r5s22}; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/splendor-rl-gym_amd/splendor_amd/variants
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
for L in default dagg0 parts8; do
    unset SPLENDOR_BEAM_LIB SB_DIST_PARTS
    [ $L = dagg0 ] && export SPLENDOR_BEAM_LIB=$V/lib_dagg0.so
    [ $L = parts8 ] && export SB_DIST_PARTS=8
    bash profiles/collect_r3_sharded.sh $O/kh_$L 8 29 5 || exit 1
    python3 profiles/sharded_table.py $O/kh_$L --world 8 --steps 5 --out $O/kh_${L}_table.json > $O/kh_${L}_table.txt
    cp $O/kh_$L/bench_r0.json $O/kh_${L}_bench_r0.json
    python3 -c "import json; d=json.load(open('$O/kh_${L}_table.json')); k=d['robust_per_kernel_ms']; m=d['robust_mean_ms']; print('$L', 'k_dest', round(k.get('k_dest',0),3), 'rebalance', round(m['rebalance partition'],3), 'expand', round(m['expand'],3), 'claims', round(m['owner claims'],3), 'device', round(m['device total (engine stream)'],3))"
    rm -rf $O/kh_$L/r*/
done
unset SB_DIST_PARTS
python3 profiles/project_n8.py $O/kh_default_table.json $O/kh_default_bench_r0.json | grep "B=  400"
python3 profiles/project_n8.py $O/kh_parts8_table.json $O/kh_parts8_bench_r0.json --parts 8 --rounds 24 | grep "B=  400"
