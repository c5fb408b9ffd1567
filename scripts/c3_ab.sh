#!/bin/bash
# C3 decimator: GPU parity (K), then bench c3 with k_decim_w4 (default) and
# k_decim_w (ORION_DECIM_W2=1), alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c3}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-decim}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "parity|passed|failed|Error|error" "$OUT/tests.log" | tail -12
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for w2 in 0 1; do
    ORION_DECIM_W2=$w2 timeout -k 10 120 python bench.py --config c3 --steps ${BSTEPS:-20} --warmup 5 --no-cpu 2>&1 | grep metric | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2=$w2', 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])" || exit 1
  done
done
