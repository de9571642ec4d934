#!/bin/bash
# Instruction-mix pass for the emission and the step's other short kernels (GPU box, repo root):
# is k_emit_w issue-bound?  SQ counters in one pass (<= 8 SQ_ per run), kernel trace in its own run.
#   profiles/valu_emit.sh OUT_DIR
set -e
OUT=${1:-gpurun_out/valu}
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="--no-cpu-baseline --steps 6 --warmup 0"
RX='k_emit|k_gather_d|k_os_pass|k_expand'
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
    --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc_sq" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_sq.json" 2> "$OUT/sq.err"
