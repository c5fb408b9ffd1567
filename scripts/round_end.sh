#!/bin/bash
# Round-end evidence: full GPU test suite, smoke, the driver's C2 command with its
# rocprofv3 kernel statistics, C3/C4/C5 lines (CPU baselines) with statistics, the
# per-block bench with statistics. The first crash/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-end}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; grep -E "^\.*\[parity\]|passed|failed" "$OUT/tests.log" | sed 's/^\.*//' > "$OUT/parity.txt"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
TAG=${TAG:-end} bash scripts/final_session.sh || exit $?
TAG=${TAG:-end} bash scripts/blocks_session.sh || exit $?
timeout -k 10 300 python tools/mod_bench.py > "gpurun_out/${TAG:-end}/mod.jsonl" 2>&1 || { tail -3 "gpurun_out/${TAG:-end}/mod.jsonl"; exit 1; }
grep -h case "gpurun_out/${TAG:-end}/mod.jsonl" | cut -c1-150
if [ "${TRAFFIC:-0}" = 1 ]; then
  TAG=${TAG:-end}_traffic CFGS="${TCFGS:-c2 c5}" bash scripts/traffic_session.sh || exit $?
fi
