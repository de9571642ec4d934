#!/bin/bash
# Round 6, session 5: host metadata latency on the GPU box's CPUs (world 8, no GPU); the same-workload N=1 references the
# N>1 bench lines carry (single-GPU engine and the sharded world-1 protocol, -H efficiency at 4M); a --gpus 2 line (gloo
# transport, both ranks on this one GPU); the W=4M and C5 world-8 sharded goldens with block-cyclic slices; the
# serialised world-8 per-rank table and the projection
O=${1:-gpurun_out/r6s5}; mkdir -p $O profiles/r6
export TMPDIR=/tmp
timeout -k 10 300 python3 profiles/gloo_latency.py --world 8 --rounds 300 --out $O/gloo_latency_w8_box.json > $O/gloo.log 2>&1 || exit 1
grep -A2 "chain" $O/gloo.log | head -4
timeout -k 10 300 python3 bench.py --gpus 1 --heuristic efficiency --no-cpu-baseline --steps 20 --warmup 5 > $O/n1_efficiency.json 2> $O/n1_efficiency.err || exit 1
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/n1_sharded_efficiency.json 2> $O/n1_sharded_efficiency.err || exit 1
cp $O/n1_efficiency.json $O/n1_sharded_efficiency.json profiles/r6/
SB_DIST_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --no-cpu-baseline --steps 6 --warmup 1 > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err || exit 1
python3 -c "
import json
for f in ('n1_efficiency', 'n1_sharded_efficiency', 'bench_g2_gloo'):
    d = json.loads(open('$O/' + f + '.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d.get('scaling_efficiency'), d.get('config', {}).get('shared_gpu'))"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 3 $O/big.log; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|record pack|device total|expand"
cp $O/t8/bench_r0.json $O/t8_bench_r0.json
python3 profiles/project_n8.py $O/t8_table.json $O/t8_bench_r0.json --host-lat-json $O/gloo_latency_w8_box.json | grep -E "B=  400|exchange per rank"
rm -rf $O/t8/r*/
