#!/bin/bash
# Scan-family ablations: block rows per experiment build (EXP: names under
# orion-sdr_amd/exp, "base" = lib/), ROWS: block_bench rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abl}; mkdir -p "$OUT"
for e in ${EXP:-base}; do
  if [ "$e" = base ]; then L=$PWD/orion-sdr_amd/lib/liborion_sdr_amd.so; else L=$PWD/orion-sdr_amd/exp/$e/liborion_sdr_amd.so; fi
  ORION_SDR_LIB=$L timeout -k 10 200 python tools/block_bench.py --no-cpu --rows "${ROWS:-a6,a7,a9,a10,a11,a12}" > "$OUT/$e.jsonl" 2>&1 || { tail -3 "$OUT/$e.jsonl"; exit 1; }
  echo "== $e"; grep -o '"row": "[a-z0-9]*", "block": "[^"]*", "n": [0-9]*, "ms_per_call": [0-9.]*' "$OUT/$e.jsonl" | sed 's/"n": [0-9]*, //'
done
