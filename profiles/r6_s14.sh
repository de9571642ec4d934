#!/bin/bash
# Round 6, session 14: two exchange parts per turn against four — the sharded GPU suite and the W=4M / C5 world-8 goldens
# with SB_DIST_PARTS=2 as the default, the world-1 key-pass run at P = 2 / 3 / 4 (interleaved), the serialised world-8
# table at P = 2 and its projection
O=${1:-gpurun_out/r6s14}; mkdir -p $O
export TMPDIR=/tmp
export SB_DIST_PARTS=2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 2 $O/big.log; [ $rc -eq 0 ] || exit $rc
kp1() {   # name, parts
    SB_DIST_PARTS=$2 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$1.json 2> $O/kp1_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$1.json')); print('kp1 $1', round(d['value']/1e6,1), d['ms_per_step'])"
}
kp1 p2_1 2 && kp1 p3_1 3 && kp1 p4_1 4 && kp1 p2_2 2 && kp1 p3_2 3 && kp1 p4_2 4 || exit 1
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|joint select|rebalance|device total|expand"
cp $O/t8/bench_r0.json $O/t8_bench_r0.json
python3 profiles/project_n8.py $O/t8_table.json $O/t8_bench_r0.json --host-lat-json profiles/r6/s5/gloo_latency_w8_box.json --single-ms 4.451 --parts 2 | grep -E "B=  400|exchange per rank"
rm -rf $O/t8/r*/
