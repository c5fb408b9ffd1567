#!/bin/bash
# GPU iteration: a pytest -k subset (K), then the driver's C2 bench command.
#   K="rotator or wbfm" TAG=x bash scripts/gpu_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-chk}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 ${TT:-600} python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread -k "${K:-wbfm}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "^\[parity\]|passed|failed|Error" "$OUT/tests.log" | tail -${NL:-40}
[ $rc -le 1 ] || exit $rc
[ "${BENCH:-1}" = 1 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
cut -c1-400 "$OUT/bench.json"
exit $rc
