#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pf1b}; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$PWD/orion-sdr_amd/lib/abl/liborion_x95.so
ORION_SDR_LIB=$LIB AB_ROUNDS=16 timeout -k 10 300 python tools/ab_paths.py segmented4@95,segmented4 c2 2>&1 | grep median || exit 1
ORION_SDR_LIB=$LIB AB_ROUNDS=16 timeout -k 10 300 python tools/ab_paths.py segmented4,segmented4@95 c4 2>&1 | grep median || exit 1
for rep in 1 2 3; do
  for v in 95 31; do
    ORION_SDR_LIB=$LIB ORION_SEG4_X=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/b_${v}_$rep.log 2>&1 || exit 1
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if 'metric' in l][-1]);print('X=$v', d['value'], d['roofline']['kernel_ms'])" $OUT/b_${v}_$rep.log
  done
done
