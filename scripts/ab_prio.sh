#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in q6 q12; do
  echo "== $v"
  ORION_SDR_LIB=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so AB_ROUNDS=16 timeout -k 10 300 python tools/ab_paths.py segmented4,segmented4@223 c2 2>&1 | grep median || exit 1
done
