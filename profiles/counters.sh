#!/bin/bash
# PMC counter passes (one rocprofv3 run per group, --pmc only with kernel filtering) for the bench
# workload; run on the GPU box from the repo root.  Output: $OUT/<group>/run_counter_collection.csv
set -e
OUT=${1:-gpurun_out/pmc}
KRE=${2:-'k_expand|k_emit|k_sel|k_sort|k_gather'}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" --output-format csv -d "$OUT/$name" -o run -- \
        python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT
run sq3 SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_FP64 SQ_ACTIVE_INST_VALU
run tcc TCC_HIT_sum TCC_MISS_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
