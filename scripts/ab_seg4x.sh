#!/bin/bash
# In-process A/B of k_wbfm_seg4 variants (tools/ab_paths.py "segmented4@<bits>"), plus
# optional abl libs ($VARS); parity of the alternate variant first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
if [ -n "${XT:-}" ]; then
  ORION_SEG4_X=$XT timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "wbfm" > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
fi
AB_ROUNDS=${R:-16} timeout -k 10 300 python tools/ab_paths.py ${PATHS:-segmented4,segmented4@3} c2 2>&1 | grep median || exit 1
for v in ${VARS:-}; do
  echo "== $v"
  ORION_SDR_LIB=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so AB_ROUNDS=${R:-16} timeout -k 10 300 python tools/ab_paths.py ${VPATHS:-segmented4,segmented4@3} c2 2>&1 | grep median || exit 1
done
