set -u
OUT=gpurun_out/${TAG:-r5c}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wbfm_exp.py --multi --rounds 4 --k 20 ${VARIANTS} > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
tail -12 $OUT/ab.txt
if [ -n "${K:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K}" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -E "^\.*\[parity\]|passed|failed" $OUT/tests.log | sed 's/^\.*//' > $OUT/parity.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ "${RT:-0}" = 1 ]; then timeout -k 10 300 python -u tools/roundtrip_bench.py ${RTARGS:-} > $OUT/rt.jsonl 2>&1 || { tail -5 $OUT/rt.jsonl; exit 1; }; cut -c1-400 $OUT/rt.jsonl; fi
