#!/bin/bash
# seg3 bring-up: parity on the new path, then A/B timing against seg2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-s3}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-segmented3}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "parity|passed|failed|Error|error" "$OUT/tests.log" | tail -30
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/ab_paths.py ${PATHS:-segmented,segmented3} 2>&1 | grep -v amdgpu.ids
