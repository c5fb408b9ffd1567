set -u
OUT=gpurun_out/r5a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; grep -E "^\.*\[parity\]|passed|failed" $OUT/tests.log | sed 's/^\.*//' > $OUT/parity.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c2.log 2>&1; tail -1 $OUT/c2.log
