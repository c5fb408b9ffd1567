#!/bin/bash
# Timing variants of the engine (orion-sdr_amd/lib/abl/liborion_<tag>.so, $VARS):
# per lib an interleaved-round timing (tools/ab_paths.py) and the seg2 phase trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-var}; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in product ${VARS:-}; do
  lib=""; [ "$v" = product ] || lib=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so
  echo "== $v"
  ORION_SDR_LIB=$lib timeout -k 10 120 python tools/ab_paths.py ${PATHS:-segmented} ${CFG:-c2} 2>&1 | grep median || exit 1
  ORION_SDR_LIB=$lib timeout -k 10 120 python tools/seg2_trace.py "$OUT/trace_$v.bin" 2>&1 | grep -E "span|early|late|IIR sub2|tail" || exit 1
done
