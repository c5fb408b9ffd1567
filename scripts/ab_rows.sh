#!/bin/bash
# Interleaved tools/block_bench.py A/B of library variants (base = lib/, others = exp/NAME), rows ROWS:
#   ROWS=a7,a10 bash scripts/ab_rows.sh   VARIANTS="base NAME" ROUNDS=2
mkdir -p gpurun_out/mp
for r in $(seq 1 "${ROUNDS:-2}"); do for v in ${VARIANTS:-base head}; do
  if [ $v = base ]; then lib=$PWD/orion-sdr_amd/lib/liborion_sdr_amd.so; else lib=$PWD/orion-sdr_amd/exp/$v/liborion_sdr_amd.so; fi
  ORION_SDR_LIB=$lib timeout -k 10 120 python tools/block_bench.py --rows ${ROWS:-a6,a7,a9,a10,a11,a12} --no-cpu > gpurun_out/mp/rows_$v$r.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/mp/rows_$v$r.jsonl'):
    d=json.loads(l); print('$r $v', d['row'], d['block'][:30], d['ms_per_call'], d['frac_of_8TBs'])"
done; done
