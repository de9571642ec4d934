#!/bin/bash
# round 3: does RCCL run two ranks on one GPU?  If so, the sharded bench over RCCL at world 2 on one GPU
O=${1:-gpurun_out/r3l}; mkdir -p $O
timeout -k 10 120 python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    profiles/probe/rccl_two_ranks_one_gpu.py > $O/probe.log 2>&1
rc=$?
grep "rank" $O/probe.log | grep -v Gloo | tail -4
echo "probe rc=$rc"
if [ $rc -ne 0 ]; then exit 0; fi
SB_DIST_SHARE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
    bench.py --gpus 2 --no-cpu-baseline --steps 6 --warmup 0 > $O/bench_rccl_w2.json 2> $O/bench_rccl_w2.err
echo "bench rc=$?"
tail -1 $O/bench_rccl_w2.json
