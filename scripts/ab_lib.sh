#!/bin/bash
# Change check against timing variants of the engine: GPU parity (K) on the
# product lib, then tools/ab_paths.py per lib (product, then each
# orion-sdr_amd/lib/abl/liborion_<tag>.so in $VARS), alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-wbfm}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|Error|error" "$OUT/tests.log" | tail -8
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  echo "== product"
  timeout -k 10 120 python tools/ab_paths.py ${PATHS:-segmented} ${CFG:-c2} 2>&1 | grep median || exit 1
  for v in ${VARS:-}; do
    echo "== $v"
    ORION_SDR_LIB=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so timeout -k 10 120 python tools/ab_paths.py ${PATHS:-segmented} ${CFG:-c2} 2>&1 | grep median || exit 1
  done
done
