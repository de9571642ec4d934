#!/bin/bash
# Round 6, session 21: the key pass hashes a batch's buys in rounds of their own into LDS and walks the records in
# order for takes, owners and ranks (SB_KS_BUYQ, default) — sharded GPU parity + W=4M / C5 world-8 goldens, the
# expansion micro-bench and the world-1 key-pass run against the SB_KS_BUYQ=0 build, the serialised world-8 table
O=${1:-gpurun_out/r6s21}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 2 $O/big.log; [ $rc -eq 0 ] || exit $rc
D=splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so
timeout -k 10 240 python3 profiles/expand_bench.py --turn 11 --reps 3 > $O/eb_buyq.json 2> $O/eb_buyq.err || exit 1
SPLENDOR_BEAM_LIB=ab/libsb_nobuyq.so timeout -k 10 240 python3 profiles/expand_bench.py --turn 11 --reps 3 > $O/eb_nobuyq.json 2> $O/eb_nobuyq.err || exit 1
for f in buyq nobuyq; do python3 -c "
import json; d=json.load(open('$O/eb_$f.json'))
print('$f', {k: d[k] for k in ('keys_a_no_own','dbg_a_no_claims','dbg_a_no_claims_cheap_key','dbg_a_no_claims_no_stores','keypass_a_w8')})"; done
kp1() {   # name, lib
    SPLENDOR_BEAM_LIB=$2 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$1.json 2> $O/kp1_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/kp1_$1.json')); print('kp1 $1', round(d['value']/1e6,1), d['ms_per_step'])"
}
kp1 buyq_1 $D && kp1 nobuyq_1 ab/libsb_nobuyq.so && kp1 buyq_2 $D && kp1 nobuyq_2 ab/libsb_nobuyq.so || exit 1
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|joint select|rebalance|device total|expand|per kernel"
cp $O/t8/bench_r0.json $O/t8_bench_r0.json
python3 profiles/project_n8.py $O/t8_table.json $O/t8_bench_r0.json --host-lat-json profiles/r6/s5/gloo_latency_w8_box.json --single-ms 4.451 | grep -E "latency|B=  400"
rm -rf $O/t8/r*/
