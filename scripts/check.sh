#!/bin/bash
# GPU check after a change: the full -m gpu suite, then the driver's C2 bench
# command and a C1 line. The first failure (or a time limit) ends the session.
#   TAG=x bash scripts/check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-check}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ${PYARGS:-} > "$OUT/tests.log" 2>&1
rc=$?; tail -15 "$OUT/tests.log"; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_c2.json" 2>&1 || { tail -5 "$OUT/bench_c2.json"; exit 1; }
grep metric "$OUT/bench_c2.json" | cut -c1-400
timeout -k 10 300 python bench.py --config c1 --steps 30 --warmup 3 > "$OUT/bench_c1.json" 2>&1 || { tail -5 "$OUT/bench_c1.json"; exit 1; }
grep metric "$OUT/bench_c1.json" | cut -c1-600
