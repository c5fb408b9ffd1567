#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-scanw3}; mkdir -p "$OUT"; export TMPDIR=/tmp
ORION_SDR_LIB=$PWD/orion-sdr_amd/lib/abl/liborion_w3.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "single_pass or lp_cascade or fm_demod or pm_ssb" > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in prod w3; do
    L=""; [ $v = prod ] || L=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so
    ORION_SDR_LIB=$L timeout -k 10 120 python tools/block_bench.py --cpu-n 4096 > "$OUT/$v.jsonl" 2>&1 || { tail -3 "$OUT/$v.jsonl"; exit 1; }
    grep -E '"a6"|"a9"|"a12"' "$OUT/$v.jsonl" | python3 -c "import sys,json;[print('$v',(d:=json.loads(l))['block'][:30],d['ms_per_call']) for l in sys.stdin]"
  done
done
