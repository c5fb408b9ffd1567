#!/bin/bash
# Quick GPU iteration: WBFM parity tests, then the bench under rocprofv3 kernel
# trace (per-kernel average), then the bench's own JSON line.
#   K="wbfm or ssb" TAG=q bash scripts/quick.sh   (K: a pytest -k expression)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-q}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-wbfm}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "parity|passed|failed|Error|error" "$OUT/tests.log" | tail -25
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu ${BARGS:-} > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 scripts/prof_summary.py "$OUT/prof" | grep avg; rm -rf "$OUT/prof"
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BARGS:-} 2>&1 | grep metric | tee "$OUT/bench.json"
