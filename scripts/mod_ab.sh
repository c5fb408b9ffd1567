#!/bin/bash
# Modulator parity, then tools/mod_bench.py on the product library vs $VARS libraries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-modab}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "mod" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "ssb|passed|failed|Error" "$OUT/tests.log" | tail -10; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in prod ${VARS:-t0}; do
    L=""; [ $v = prod ] || L=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so
    ORION_SDR_LIB=$L timeout -k 10 120 python tools/mod_bench.py > "$OUT/$v.jsonl" 2>&1 || { tail -3 "$OUT/$v.jsonl"; exit 1; }
    grep Ssb "$OUT/$v.jsonl" | cut -c1-120 | sed "s/^/$v /"
  done
done
