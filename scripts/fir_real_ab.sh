#!/bin/bash
# k_fir_real8 check: FIR / chain parity, then FirLowpass timing vs ORION_FIR_REAL2=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-firab}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "fir_lowpass or graph or chain or overlap" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "fir 125|fir .* taps|passed|failed|Error" "$OUT/tests.log" | tail -14; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
  ORION_FIR_REAL2=$v timeout -k 10 120 python tools/block_bench.py --cpu-n 4096 > "$OUT/b$v.jsonl" 2>&1 || { tail -3 "$OUT/b$v.jsonl"; exit 1; }
  grep '"a3"' "$OUT/b$v.jsonl" | sed "s/^/REAL2=$v /" | cut -c1-160
done
