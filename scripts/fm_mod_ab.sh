#!/bin/bash
# k_fm_mod_sp check: modulator parity, then tools/mod_bench.py single pass vs ORION_FM_MOD_3P=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-fmab}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "mod or roundtrip or round_trip" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "fm|passed|failed|Error" "$OUT/tests.log" | tail -14; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
  ORION_FM_MOD_3P=$v timeout -k 10 120 python tools/mod_bench.py > "$OUT/m$v.jsonl" 2>&1 || { tail -3 "$OUT/m$v.jsonl"; exit 1; }
  grep -E "Fm|round" "$OUT/m$v.jsonl" | sed "s/^/3P=$v /" | cut -c1-170
done
