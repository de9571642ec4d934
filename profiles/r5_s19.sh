#!/bin/bash
# Round 5, session 19: every part's own records land in the receive buffer by a device copy on the claim stream
# instead of the all_to_all (RCCL copied them at 0.4 TB/s: 1.8-2.0 ms per step at world 1): sharded parity (incl.
# RCCL's device-side completion contract and the W=4M / C5 world-8 goldens), the world-1 key-pass measurement, the
# serialised world-8 table
O=${1:-gpurun_out/r5s19}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 600 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -1 $O/big.log; [ $rc -eq 0 ] || exit $rc
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_kp1 -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_kp1.json 2> $O/tr_kp1.err || exit 1
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --top 14 | tail -3
python3 profiles/busy_union.py $O/tr_kp1 --skip 24 --exclude 'rccl|k_mt_' | tail -1
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|record pack|device total"
cp $O/t8/bench_r0.json $O/t8_bench_r0.json
python3 profiles/project_n8.py $O/t8_table.json $O/t8_bench_r0.json | grep "B=  400"
rm -rf $O/t8/r*/
