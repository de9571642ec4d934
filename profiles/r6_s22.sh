#!/bin/bash
# Round 6, session 22: the N>1 bench path on the final tree, two ranks sharing the one GPU over gloo (RCCL refuses two
# ranks on one device): bench.py's own launcher, and the driver's torch.distributed.run form (LOCAL_WORLD_SIZE set, so
# the host metadata goes over shared memory)
O=${1:-gpurun_out/r6s22}; mkdir -p $O
export TMPDIR=/tmp
SB_DIST_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --no-cpu-baseline --steps 6 --warmup 1 > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err || exit 1
SB_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --no-cpu-baseline --steps 6 --warmup 1 > $O/bench_g2_torchrun.json 2> $O/bench_g2_torchrun.err || exit 1
for f in bench_g2_gloo bench_g2_torchrun; do python3 -c "
import json; d=[json.loads(l) for l in open('$O/$f.json') if l.startswith('{')][-1]
print('$f', round(d['value']/1e6,2), d['ms_per_step'], d.get('scaling_efficiency'), d['config'].get('shared_gpu'), d.get('collectives_per_step_rank0'), list(d.get('n1_same_workload', {}).keys())[:4])"; done
