#!/bin/bash
# Per-launch sequence of a config's kernel: rocprofv3 kernel trace
# plus GRBM_GUI_ACTIVE per dispatch (its ratio to the dispatch's duration is the
# effective GPU clock), over STEPS back-to-back bench.py launches after no warm-up.
#   CFGS="c5 c2" STEPS=60 TAG=x bash scripts/seq_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-seq}; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in ${CFGS:-c5}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d "$OUT/$c" -o run -- python3 bench.py --config $c --steps ${STEPS:-60} --warmup 0 --no-cpu --no-h2d ${BARGS:-} > "$OUT/$c.log" 2>&1 || { echo "$c failed"; tail -5 "$OUT/$c.log"; exit 1; }
  python3 tools/seq_summary.py "$OUT/$c" > "$OUT/seq_$c${SUF:-}.txt" && tail -14 "$OUT/seq_$c${SUF:-}.txt"
  rm -rf "$OUT/$c"
done
