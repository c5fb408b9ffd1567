#!/bin/bash
# The driver's bench command (20 steps after 5 warm-up) per WBFM kernel path
# (ORION_WBFM_PATH; "" = the default), alternated $REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
  for p in ${BPATHS:-"" seg seg2}; do
    ORION_WBFM_PATH=$p timeout -k 10 120 python bench.py --steps ${BSTEPS:-20} --warmup 5 --no-cpu 2>&1 | grep metric | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('path=${p:-default}', 'ms_per_step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" || exit 1
  done
done
