# GPU tests selected by K (a pytest -k expression), then the paired in-process A/B of the
# working-tree library (base) against variant libraries (VARIANTS, scripts/build_variant.sh)
# on CASES (tools/ab_variants.py):
#   TAG=x K="wbfm" CASES="c2 c4" VARIANTS="base h0" ROUNDS=4 KK=10 bash scripts/tests_ab.sh
set -u
OUT=gpurun_out/${TAG:-tests_ab}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K}" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; grep -E "^\.*\[parity\]|passed|failed" $OUT/tests.log | sed 's/^\.*//' > $OUT/parity.txt
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-tests_ab} bash scripts/ab.sh
