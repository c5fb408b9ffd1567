#!/bin/bash
# HBM traffic of single blocks: FmQuadratureDemod (a9, 2^24) and
# FmPhaseAccumMod (2^26), FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes;
# tools/traffic.py OUT a9 fmmod writes profiles/traffic_<cfg>.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-trows}; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in a9 fmmod; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    if [ $c = a9 ]; then set -- tools/block_bench.py --rows a9 --no-cpu --steps 3; else set -- tools/mod_bench.py --only FmPhaseAccumMod --steps 3; fi
    timeout -s KILL 120 rocprofv3 --pmc $ctr -f csv -d "$OUT/${c}_$ctr" -o run -- python3 "$@" > "$OUT/${c}_$ctr.log" 2>&1 || { tail -5 "$OUT/${c}_$ctr.log"; exit 1; }
    f=$(find "$OUT/${c}_$ctr" -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/${c}_$ctr.csv"; rm -rf "$OUT/${c}_$ctr"
  done
done
python3 tools/traffic.py "$OUT" a9 fmmod
