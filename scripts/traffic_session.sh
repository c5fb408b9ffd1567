#!/bin/bash
# HBM traffic per launch for the bench configs: rocprofv3 --pmc FETCH_SIZE and
# --pmc WRITE_SIZE in separate passes (MI355X_MICROARCH.md: they cannot share one),
# bench.py --steps 3 --warmup 1 per pass. tools/traffic.py turns them into
# profiles/traffic_<cfg>.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-traffic}; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in ${CFGS:-c3 c4 c5}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -f csv -d "$OUT/${c}_$ctr" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --config $c > "$OUT/${c}_$ctr.log" 2>&1 || { tail -5 "$OUT/${c}_$ctr.log"; exit 1; }
    f=$(find "$OUT/${c}_$ctr" -name "*counter_collection.csv" | head -1); cp "$f" "$OUT/${c}_$ctr.csv"; rm -rf "$OUT/${c}_$ctr"
  done
done
echo "=== done"
