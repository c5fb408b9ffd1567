#!/bin/bash
# C5 (k_lpdc_sp) parity, then alternating bench runs: default lane run (kSpC) vs ORION_SP_C16=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c5ab}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-ssb or am_ or lpdc or agc or mod}" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in 0 1; do
    ORION_SP_C16=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --config c5 > "$OUT/b_${v}_${rep}.log" 2>&1 || { tail -3 "$OUT/b_${v}_${rep}.log"; exit 1; }
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if 'metric' in l][-1]);print('C16=$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/b_${v}_${rep}.log"
  done
done
