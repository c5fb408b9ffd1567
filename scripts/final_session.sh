#!/bin/bash
# Round-end measurement set: the driver's C2 command (bench line + rocprofv3 kernel
# statistics of the same command), then C1/C3/C4/C5/C5F lines with their CPU baselines and
# kernel statistics. Every GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-final}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== [$name] $*"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; grep -h metric "$OUT/$name.log" | tail -1; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }; }
# every line at the driver's own command (20 timed steps after 3 warm-ups; DESIGN §6: the
# GPU clock moves over a launch sequence, so no config gets a window of its own)
run c2 300 python bench.py
run prof_c2 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_c2" -o run -- python3 bench.py --no-cpu
for c in ${CFGS:-c1 c3 c4 c5 c5f}; do
  run $c 300 python bench.py --config $c
  run prof_$c 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$c" -o run -- python3 bench.py --no-cpu --config $c
done
for d in "$OUT"/prof_*; do f=$(find "$d" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$OUT/kernel_stats_$(basename $d | sed s/prof_//).csv"; done
rm -rf "$OUT"/prof_*/ "$OUT"/prof/ 2>/dev/null; echo "=== done"
