#!/bin/bash
# GPU check of the modulators: their tests, then tools/mod_bench.py under rocprofv3
# kernel trace and on its own.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-mod}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-mod or roundtrip}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "parity.*fm_mod|passed|failed|Error|error" "$OUT/tests.log" | tail -20
[ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/mod_bench.py > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 scripts/prof_summary.py "$OUT/prof" | grep avg | tee "$OUT/kstats.txt"; rm -rf "$OUT/prof"
timeout -k 10 180 python tools/mod_bench.py > "$OUT/mod.jsonl" 2>&1 || { tail -3 "$OUT/mod.jsonl"; exit 1; }
grep -h case "$OUT/mod.jsonl" | cut -c1-200
