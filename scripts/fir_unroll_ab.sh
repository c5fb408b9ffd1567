#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-firu}; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for v in prod u2 u4; do
    L=""; [ $v = prod ] || L=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so
    ORION_SDR_LIB=$L timeout -k 10 120 python tools/block_bench.py --cpu-n 4096 > "$OUT/$v.jsonl" 2>&1 || { tail -3 "$OUT/$v.jsonl"; exit 1; }
    grep -E '"a3"|"a5"' "$OUT/$v.jsonl" | python3 -c "import sys,json;[print('$v',(d:=json.loads(l))['row'],d['ms_per_call'],d['frac_of_8TBs']) for l in sys.stdin]"
  done
done
