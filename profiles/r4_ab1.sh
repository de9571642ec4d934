#!/bin/bash
# Round 4: single-GPU A/B of library builds on C3 (bench.py, two interleaved rounds): step time and phases
#   bash profiles/r4_ab1.sh OUT_DIR LIB1 LIB2 ...   (LIB "default" = the in-tree build)
O=${1:-gpurun_out/r4ab1}; shift; mkdir -p $O
for round in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$lib; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 12 --warmup 2 > $O/${name}_$round.json 2> $O/${name}_$round.err || { echo "$name failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${name}_$round.json').read().strip().splitlines()[-1]); print('$name', $round, round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms', d.get('phases_ms'))"
  done
done
