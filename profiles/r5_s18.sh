#!/bin/bash
# Round 5, session 18: why k_claim_goc takes 2.85-3.05 ms in a world-1 key-pass run (one shard on the GPU) against
# 3.76-4.03 ms in the serialised world-8 traces (eight processes' shards on one GPU): the world-1 run with the
# world-8 runs' shard size (visited_log2 29) and with the automatic one, same box, kernel traces
O=${1:-gpurun_out/r5s18}; mkdir -p $O
export TMPDIR=/tmp
for VL in 29 0; do
    SB_FORCE_DIST=1 SB_DIST_KP1=1 SB_VISITED_LOG2=$VL timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $O/tr_vl$VL -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_vl$VL.json \
        2> $O/tr_vl$VL.err || exit 1
    echo "visited_log2 $VL:"
    python3 profiles/busy_union.py $O/tr_vl$VL --skip 24 --exclude 'rccl|k_mt_' --top 6 | tail -2
    grep -E "visited|log2" $O/tr_vl$VL.err | head -3
done
bash profiles/collect_r3_sharded.sh $O/t8 8 29 5 || exit 1
python3 profiles/sharded_table.py $O/t8 --world 8 --steps 5 --out $O/t8_table.json | grep -E "owner claims|device total|per kernel"
rm -rf $O/t8/r*/
