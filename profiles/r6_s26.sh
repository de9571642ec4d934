#!/bin/bash
# Round 6, session 26: the key pass's per-part ticket clears and the unused own-lost clear (global-order claims) gone
# from the engine stream ahead of the parts — sharded GPU parity + W=4M / C5 world-8 goldens, the world-1 run twice
O=${1:-gpurun_out/r6s26}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/dist.log 2>&1
rc=$?; tail -n 2 $O/dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_big.py -x -v -k "w4m or world8" --timeout 800 --timeout-method thread > $O/big.log 2>&1
rc=$?; tail -n 2 $O/big.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_$i.json 2> $O/kp1_$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/kp1_$i.json')); print('kp1 $i', round(d['value']/1e6,1), d['ms_per_step'])"
done
