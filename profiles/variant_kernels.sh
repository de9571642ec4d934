#!/bin/bash
# Kernel trace of bench.py for every built variant (profiles/variants.py build ...); prints the mean
# duration of the kernels matching $1 per variant.  GPU box, repo root: bash profiles/variant_kernels.sh REGEX
set -e
RE=${1:-k_os_hist}
export TMPDIR=/tmp
for f in splendor-rl-gym_amd/splendor_amd/variants/*.so; do
    n=$(basename "$f" .so)
    SPLENDOR_BEAM_LIB=$PWD/$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/vk/$n -o run -- python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/vk/$n.json 2> gpurun_out/vk/$n.err
    python3 - "$n" "$RE" <<'P'
import csv, re, sys
n, rx = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(f'gpurun_out/vk/{n}/run_kernel_stats.csv')))
for r in rows:
    if re.search(rx, r['Name']):
        print(f"{n:14s} {r['Name'][:40]:40s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us", flush=True)
P
done
