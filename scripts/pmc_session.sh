#!/bin/bash
# PMC passes on bench.py (one rocprofv3 run per counter set, each under its own
# time limit); prints the per-dispatch means of our kernels.
#   SETS="A B C;D E" TAG=x BARGS=... bash scripts/pmc_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
IFS=';' read -ra SS <<< "$SETS"
for set in "${SS[@]}"; do
  i=$((i+1))
  timeout -k 10 90 rocprofv3 --pmc $set -d "$OUT/p$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BARGS:-} > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 scripts/prof_summary.py "$OUT" | tee "$OUT/summary.txt"; rm -rf "$OUT"/p[0-9]*/
