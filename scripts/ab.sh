set -u
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT; export TMPDIR=/tmp
for c in ${CASES}; do
  timeout -k 10 300 python -u tools/ab_variants.py --case $c --rounds ${ROUNDS:-4} --k ${KK:-10} ${VARIANTS} > $OUT/ab_$c.txt 2>&1 || { tail -5 $OUT/ab_$c.txt; exit 1; }
  echo "== $c"; tail -$(( $(echo ${VARIANTS} | wc -w) * 2 + 1 )) $OUT/ab_$c.txt
done
