#!/bin/bash
# bench.py (--config $CFG, 20 steps after 5 warm-up) per engine build: the product
# lib, then each orion-sdr_amd/lib/abl/liborion_<tag>.so in $VARS, alternated $REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
  for v in product ${VARS:-}; do
    lib=""; [ "$v" = product ] || lib=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so
    ORION_SDR_LIB=$lib timeout -k 10 120 python bench.py --config ${CFG:-c2} --steps ${BSTEPS:-20} --warmup 5 --no-cpu 2>&1 | grep metric | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])" || exit 1
  done
done
