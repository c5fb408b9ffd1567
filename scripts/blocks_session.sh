#!/bin/bash
# Per-block (§8(a) rows) throughput lines and their kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-blocks}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python tools/block_bench.py > "$OUT/blocks.jsonl" 2> "$OUT/blocks.err" || { tail -5 "$OUT/blocks.err"; exit 1; }
cat "$OUT/blocks.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 tools/block_bench.py --cpu-n 65536 > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_blocks.csv"
rm -rf "$OUT"/prof_*/ "$OUT"/prof/ 2>/dev/null; echo "=== done"
