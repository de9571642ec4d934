#!/bin/bash
# Round 4: A/B of k_mkeys_a builds (profiles/variants.py build ...) on the card-set protocol, world 2 on ONE GPU,
# serialised ranks (each rank's kernels alone on the device): the key pass's device time per step (HIP events,
# roofline.launch_ms of rank 0's line) and the step time, two interleaved rounds.
#   bash profiles/r4_mk_ab.sh OUT_DIR LIB1 LIB2 ...      (LIB: path of a built variant, or "default")
O=${1:-gpurun_out/r4ab}; shift; mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    PORT=$((20000 + RANDOM % 20000)); pids=()
    for r in 0 1; do
      if [ "$lib" = default ]; then unset SPLENDOR_BEAM_LIB; else export SPLENDOR_BEAM_LIB=$lib; fi
      RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
      SB_DIST_BACKEND=gloo SB_DIST_SERIALIZE=1 SB_DIST_FLAGS=257 \
      timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu-baseline --steps 6 --warmup 0 \
          > $O/${name}_$round.r$r.json 2> $O/${name}_$round.r$r.err &
      pids+=($!)
    done
    rc=0; for p in "${pids[@]}"; do wait $p || rc=$?; done
    [ $rc -eq 0 ] || { echo "$name round $round failed rc=$rc"; tail -5 $O/${name}_$round.r0.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open('$O/${name}_$round.r0.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', $round, 'key pass', r.get('launch_ms'), 'ms/step; step', d['ms_per_step'], 'ms; frac', r.get('frac'))"
  done
done
