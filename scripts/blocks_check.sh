#!/bin/bash
# GPU check of the per-block rows: the GPU tests matching K, then tools/block_bench.py
# (small CPU sample) under rocprofv3 kernel trace and on its own.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-blk}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-scan or lp_cascade or fm_demod or pm_ssb or biquad or geometry}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|Error|error" "$OUT/tests.log" | tail -8
[ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/block_bench.py --cpu-n ${CPUN:-65536} > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 scripts/prof_summary.py "$OUT/prof" | grep avg | tee "$OUT/kstats.txt"; rm -rf "$OUT/prof"
timeout -k 10 240 python tools/block_bench.py --cpu-n ${CPUN:-65536} > "$OUT/blocks.jsonl" 2>&1 || { tail -3 "$OUT/blocks.jsonl"; exit 1; }
python3 -c "
import json
for l in open('$OUT/blocks.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('row'), d.get('block','')[:40], d.get('ms_per_call'), d.get('frac_of_8TBs', d.get('frac')))
"
