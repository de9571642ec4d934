#!/bin/bash
# round 3, session 5: engine parity + smoke on the final tree, then per-kernel traces of the select's grid /
# loads-in-flight knobs (select histogram grid 256/512/1024, 8 or 16 loads per thread; stage grid 1024/2048/4096)
O=${1:-gpurun_out/s5n}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_realistic.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
bash profiles/r3s5_trace_variants.sh $O/trace > $O/trace.txt 2>&1 || exit $?
grep -E "lib_|k_tk_hist|k_tk_stage|k_tk_unstage|k_tk_count|k_tk_write" $O/trace.txt
