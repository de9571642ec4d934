#!/bin/bash
# round 3: C5 parity at its own width (single GPU W=32M; sharded world 8 on one GPU), then sharded traces
O=${1:-gpurun_out/r3c}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_big.py -k c5 -x -v --timeout 900 --timeout-method thread > $O/tests_c5.log 2>&1
rc=$?
tail -3 $O/tests_c5.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash profiles/r3_run_sharded.sh $O
