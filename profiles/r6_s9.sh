#!/bin/bash
# Round 6, session 9: the key pass's count scan in k_keys_a's last workgroup (no scan / counts / copy launches behind
# each part on the engine stream), the parts' claim tickets cleared once per turn: sharded GPU parity + W=4M / C5
# world-8 goldens, KP1 A/B (tail scan on / off, claims grid 2048 / 1024), kernel + HIP runtime trace of the KP1 step,
# the serialised world-8 per-rank table and the projection
O=${1:-gpurun_out/r6s9}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 2 $O/big.log; [ $rc -eq 0 ] || exit $rc
kp1() {   # name, env...
    local n=$1; shift
    env "$@" SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$n.json 2> $O/kp1_$n.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$n.json')); print('kp1 $n', round(d['value']/1e6,1), d['ms_per_step'])"
}
kp1 tail_1 SB_KS_TAIL=1 && kp1 notail_1 SB_KS_TAIL=0 && kp1 tail_g1024_1 SB_KS_TAIL=1 SB_GOC_GRID=1024 && \
kp1 tail_2 SB_KS_TAIL=1 && kp1 notail_2 SB_KS_TAIL=0 && kp1 tail_g1024_2 SB_KS_TAIL=1 SB_GOC_GRID=1024 || exit 1
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/tr_kp1 -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_kp1.json 2> $O/tr_kp1.err || exit 1
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --top 16 | tail -2
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --exclude 'rccl|k_mt_' | tail -1
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|joint select|rebalance|device total|expand"
cp $O/t8/bench_r0.json $O/t8_bench_r0.json
python3 profiles/project_n8.py $O/t8_table.json $O/t8_bench_r0.json --host-lat-json profiles/r6/s5/gloo_latency_w8_box.json | grep -E "B=  400|exchange per rank"
rm -rf $O/t8/r*/
