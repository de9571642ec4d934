set -e
OUT=gpurun_out/r2u; mkdir -p $OUT
for f in splendor-rl-gym_amd/splendor_amd/variants/lib_*.so; do
  echo "== $f" >> $OUT/sortbench.txt
  SPLENDOR_BEAM_LIB=$PWD/$f timeout -k 10 120 python3 -u profiles/sortbench.py >> $OUT/sortbench.txt 2>&1
done
for r in 1 2; do timeout -k 10 400 python3 -u profiles/variants.py bench --steps 12 >> $OUT/ab.txt 2>&1; done
cat $OUT/sortbench.txt $OUT/ab.txt
