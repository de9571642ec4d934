#!/bin/bash
# Round 4: top-k sort digit/tile variants, C3 then C4 (bench lines, two interleaved rounds each)
#   bash profiles/r4_sort_ab.sh OUT_DIR LIB1 LIB2 ...
O=${1:-gpurun_out/r4sort}; shift; mkdir -p $O
for cfg in c3 c4; do
  extra=""; [ $cfg = c4 ] && extra="--realistic"
  for round in 1 2; do
    for lib in "$@"; do
      name=$(basename "$lib" .so)
      if [ "$lib" = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$lib; fi
      timeout -k 10 300 python3 bench.py $extra --no-cpu-baseline --steps 12 --warmup 2 > $O/${cfg}_${name}_$round.json 2> $O/${cfg}_${name}_$round.err || { echo "$cfg $name failed"; tail -3 $O/${cfg}_${name}_$round.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${cfg}_${name}_$round.json').read().strip().splitlines()[-1]); p=d['phases_ms']; print('$cfg', '$name', $round, round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms select', p.get('ms_select'), 'sort', p.get('ms_sort'))"
    done
  done
done
