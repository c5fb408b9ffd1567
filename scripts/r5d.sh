# Scan-family experiment session: the scan tests (K filter), then paired A/B of the
# working-tree library (base) against variants (VARIANTS) on CASES.
set -u
OUT=gpurun_out/${TAG:-r5d}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K}" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; grep -E "^\.*\[parity\]|passed|failed" $OUT/tests.log | sed 's/^\.*//' > $OUT/parity.txt
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r5d} bash scripts/ab.sh
