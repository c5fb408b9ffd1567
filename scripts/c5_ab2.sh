#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c5ab2}; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in prod ${VARS:-w3}; do
    L=""; [ $v = prod ] || L=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so
    ORION_SDR_LIB=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --config ${CFG:-c5} > "$OUT/b_${v}_${rep}.log" 2>&1 || { tail -3 "$OUT/b_${v}_${rep}.log"; exit 1; }
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if 'metric' in l][-1]);print('$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/b_${v}_${rep}.log"
  done
done
