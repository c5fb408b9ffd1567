#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c3q4}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "decim" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "decim|passed|failed|Error" "$OUT/tests.log" | tail -12; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for v in 1 0; do
    ORION_DECIM_Q4=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --config c3 > "$OUT/b_${v}_${rep}.log" 2>&1 || { tail -3 "$OUT/b_${v}_${rep}.log"; exit 1; }
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if 'metric' in l][-1]);print('Q4=$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/b_${v}_${rep}.log"
  done
done
