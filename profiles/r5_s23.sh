#!/bin/bash
# Round 5, session 23: HBM traffic of a rank's key kernels with one shard on the GPU (the world-1 key-pass run,
# SB_DIST_KP1=1, C5's per-rank shape): FETCH_SIZE and WRITE_SIZE passes (each its own run), and the trace they go with
O=${1:-gpurun_out/r5s23}; mkdir -p $O
export TMPDIR=/tmp
RX='k_claim_goc|k_keys_a|k_keys_b|k_apply_w'
ENVV="SB_FORCE_DIST=1 SB_DIST_KP1=1"
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --gpus 1 --no-cpu-baseline --steps 4 --warmup 0 > $O/trace.json 2> $O/trace.err || exit 1
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv \
    -d $O/fetch -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 4 --warmup 0 > $O/fetch.json 2> $O/fetch.err || exit 1
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv \
    -d $O/write -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 4 --warmup 0 > $O/write.json 2> $O/write.err || exit 1
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
def per(kind, cname):
    f = glob.glob(f'{O}/{kind}/**/*counter_collection.csv', recursive=True)[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'].startswith(cname):
            d[r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sb::', '')].append(float(r['Counter_Value']))
    return d
fe, wr = per('fetch', 'FETCH_SIZE'), per('write', 'WRITE_SIZE')
for k in sorted(fe):
    f = sorted(fe[k])[-4:]; w = sorted(wr.get(k, [0]))[-4:]
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    print(f'{k:24s} largest dispatches: FETCH {fk/1e6:.3f} GiB-units  WRITE {wk/1e6:.3f}  hbm (2*FETCH+WRITE) KiB -> {(2*fk+wk)*1024/1e9:.2f} GB')
PY
