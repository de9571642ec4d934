#!/bin/bash
# Round 4 experiment: k_expand with parents processed grouped by grandparent (SB_XP_PERM=1) against rank order:
# correctness on the W=300k reference goldens + the C3 golden, then C3 bench A/B (two interleaved rounds)
#   bash profiles/r4_perm_ab.sh OUT_DIR LIB
O=${1:-gpurun_out/r4perm}; L=$2; mkdir -p $O
SPLENDOR_BEAM_LIB=$L timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread -k "solve or stepwise" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/r4_ab1.sh $O default $L
