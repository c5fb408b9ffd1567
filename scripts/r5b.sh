set -u
OUT=gpurun_out/${TAG:-r5b}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K}" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; grep -E "^\.*\[parity\]|passed|failed" $OUT/tests.log | sed 's/^\.*//' > $OUT/parity.txt
exit $rc
