#!/bin/bash
# Round 6, session 17: the key pass hashes a batch's buys and takes in separate rounds (SB_KS_SPLIT, default) —
# sharded GPU parity + W=4M / C5 world-8 goldens, the world-1 key-pass run against the SB_KS_SPLIT=0 build
# (interleaved twice), its kernel trace, the serialised world-8 table (collectives counted) and the projection
O=${1:-gpurun_out/r6s17}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 2 $O/big.log; [ $rc -eq 0 ] || exit $rc
kp1() {   # name, lib
    SPLENDOR_BEAM_LIB=$2 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$1.json 2> $O/kp1_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$1.json')); print('kp1 $1', round(d['value']/1e6,1), d['ms_per_step'])"
}
D=splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so
kp1 split_1 $D && kp1 nosplit_1 ab/libsb_nosplit.so && kp1 split_2 $D && kp1 nosplit_2 ab/libsb_nosplit.so || exit 1
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_kp1 -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_kp1.json 2> $O/tr_kp1.err || exit 1
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --top 16 | tail -2
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --exclude 'rccl|k_mt_' | tail -1
rm -f $O/tr_kp1/run_kernel_trace.csv
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|joint select|rebalance|device total|expand|per kernel"
cp $O/t8/bench_r0.json $O/t8_bench_r0.json
python3 profiles/project_n8.py $O/t8_table.json $O/t8_bench_r0.json --host-lat-json profiles/r6/s5/gloo_latency_w8_box.json --single-ms 4.451 | grep -E "latency|B=  400|exchange per rank"
rm -rf $O/t8/r*/
