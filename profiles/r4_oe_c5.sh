#!/bin/bash
# Round 4: C5 at world 8 on one GPU, card-set ownership with and without owner emission (one pytest process each)
O=${1:-gpurun_out/r4oe5}; mkdir -p $O
nvidia-smi >/dev/null 2>&1; rocm-smi --showmeminfo vram > $O/vram_before.txt 2>&1
timeout -k 10 600 python3 -u -m pytest "tests/test_gpu_big.py::test_c5_sharded_world8_oracle_golden[oe]" -x -v --timeout 550 --timeout-method thread > $O/c5_oe.log 2>&1
rc=$?; tail -3 $O/c5_oe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest "tests/test_gpu_big.py::test_c5_sharded_world8_oracle_golden[True]" -x -v --timeout 550 --timeout-method thread > $O/c5_mig.log 2>&1
rc=$?; tail -3 $O/c5_mig.log; exit $rc
