#!/bin/bash
# The driver's own bench command (BENCH_r0*.json "cmd"), REPS times back to back on one
# box, then one rocprofv3 kernel-statistics run of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-drv}; mkdir -p "$OUT"; export TMPDIR=/tmp
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/c2_$i.json" 2> "$OUT/c2_$i.err" || { tail -5 "$OUT/c2_$i.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c2_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('run $i', d['value'], d['ms_per_step'], r['frac'], r['per_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_c2.csv"; rm -rf "$OUT/prof"
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats_c2.csv')):
    if 'wbfm' in r['Name']: print(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3)
"
