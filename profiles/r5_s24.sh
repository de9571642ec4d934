#!/bin/bash
# Round 5, session 24: does sharing the GPU with other ranks' shards slow the claims?  k_claim_goc's time and HBM
# traffic per launch with two serialised ranks on one GPU (key ownership, C5's per-rank shape), beside the one-shard
# world-1 run (session 23: 19.2 GB per launch, 3.3-4.0 ms) and the eight-rank tables (3.6-4.0 ms)
O=${1:-gpurun_out/r5s24}; mkdir -p $O
export TMPDIR=/tmp
N=2
run_pass() {   # name, rocprofv3 args...
    local name=$1; shift
    local PORT=$((20000 + RANDOM % 20000)) pids=() rc=0
    mkdir -p $O/$name
    for r in 0 1; do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        SB_DIST_BACKEND=gloo SB_DIST_SERIALIZE=1 SB_BENCH_PROGRESS=1 SB_DIST_FLAGS=32 \
        timeout -k 10 -s KILL 400 rocprofv3 "$@" --output-format csv -d $O/$name/r$r -o run -- \
            python3 bench.py --gpus $N --no-cpu-baseline --steps 4 --warmup 0 > $O/$name/bench_r$r.json 2> $O/$name/r$r.err &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait "$p" || rc=$?; done
    return $rc
}
run_pass trace --kernel-trace || exit 1
run_pass fetch --pmc FETCH_SIZE --kernel-include-regex 'k_claim_goc' || exit 1
run_pass write --pmc WRITE_SIZE --kernel-include-regex 'k_claim_goc' || exit 1
python3 - "$O" <<'PY'
import csv, glob, sys
O = sys.argv[1]
t = []
for f in glob.glob(f'{O}/trace/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_claim_goc' in r['Kernel_Name']:
            t.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
t.sort()
print('k_claim_goc world 2 serialised, largest launches (ms):', [round(x, 3) for x in t[-6:]])
for kind, cn in (('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE')):
    v = []
    for f in glob.glob(f'{O}/{kind}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'].startswith(cn):
                v.append(float(r['Counter_Value']))
    v.sort()
    print(cn, 'largest launches (KiB):', [round(x / 1e6, 3) for x in v[-6:]], 'e6')
PY
