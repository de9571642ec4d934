#!/bin/bash
# Round 5, session 17: one rank's sharded device work measured with its streams overlapping.  The world > 1
# key-owner path (pipelined key pass in 4 parts, packs on the claim stream, global-order claims, apply, emission,
# joint select, grouped... at world 1: no exchange) on one GPU at C5's per-rank shape (W=4M, efficiency), against the
# serialised world-8 table's summed kernel times.  Sharded parity first (incl. the world-1 cases).
O=${1:-gpurun_out/r5s17}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -1 $O/dist.log; [ $rc -eq 0 ] || exit $rc
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 1 \
    > $O/kp1.json 2> $O/kp1.err || exit 1
python3 -c "import json; d=json.load(open('$O/kp1.json')); print('kp1 world 1', d['ms_per_step'], 'ms/step', d.get('phases_ms'))"
SB_FORCE_DIST=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 1 \
    > $O/fused.json 2> $O/fused.err || exit 1
python3 -c "import json; d=json.load(open('$O/fused.json')); print('world-1 fused', d['ms_per_step'], 'ms/step')"
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_kp1 -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 5 --warmup 0 > $O/tr_kp1.json 2> $O/tr_kp1.err || exit 1
python3 profiles/busy_union.py $O/tr_kp1 --skip 2 | tail -8
