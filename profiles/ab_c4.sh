set -e
OUT=gpurun_out/c4ab; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 900 python3 -u profiles/variants.py bench --steps 12 --realistic >> $OUT/variants.txt 2>&1
done
cat $OUT/variants.txt
