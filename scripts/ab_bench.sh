#!/bin/bash
# Interleaved bench.py A/B of library variants (base = lib/, NAME = exp/NAME):
#   CFG=c5 ROUNDS=3 bash scripts/ab_bench.sh base c5old
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=$PWD/orion-sdr_amd/lib/liborion_sdr_amd.so; else lib=$PWD/orion-sdr_amd/exp/$v/liborion_sdr_amd.so; fi
    out=$(ORION_SDR_LIB=$lib timeout -k 10 120 python bench.py --config "${CFG:-c5}" --steps "${STEPS:-20}" --warmup 3 --no-cpu 2>/dev/null | grep metric) || { echo "$v failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('round $r', '$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel_ms'))" "$out"
  done
done
