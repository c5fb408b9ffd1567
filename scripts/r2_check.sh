#!/bin/bash
# Round-2 change check: targeted GPU parity (K), then WBFM C2 timing (rocprof
# kernel-trace average + bench line) and the TX-mask bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-chk}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-wbfm or firiq or aligned}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|Error|error" "$OUT/tests.log" | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/prof.log" 2>&1 || exit 1
python3 scripts/prof_summary.py "$OUT/prof" | grep avg
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>&1 | grep metric | cut -c1-160
timeout -k 10 120 python tools/txmask_bench.py 2>&1 | grep case | tee "$OUT/txmask.jsonl"
