#!/bin/bash
# Round-4 GPU session: the GPU tests (K: a pytest -k filter, empty = all), the C5 line,
# the driver's C2 command (+ host_fed), its rocprof kernel stats, per-block and
# modulator lines, and the WBFM A/B (AB: variant names for tools/wbfm_exp.py).
# The first crash/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread ${K:+-k "$K"} > "$OUT/tests.log" 2>&1
  rc=$?; grep -E "passed|failed|Error" "$OUT/tests.log" | tail -5; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 5 > "$OUT/bench_c5.json" 2>&1 || { tail -5 "$OUT/bench_c5.json"; exit 1; }
grep metric "$OUT/bench_c5.json" | cut -c1-300
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -5 "$OUT/bench_c2.err"; exit 1; }
cut -c1-300 "$OUT/bench_c2.json"; grep -o '"roofline".*' "$OUT/bench_c2.json" | cut -c1-900
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c2 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-h2d > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 scripts/prof_summary.py "$OUT/prof" | grep -E "k_wbfm" | head -3
timeout -k 10 300 python tools/block_bench.py > "$OUT/blocks.jsonl" 2>&1 || { tail -3 "$OUT/blocks.jsonl"; exit 1; }
timeout -k 10 300 python tools/mod_bench.py > "$OUT/mod.jsonl" 2>&1 || { tail -3 "$OUT/mod.jsonl"; exit 1; }
if [ -n "${AB:-}" ]; then
  timeout -k 10 300 python tools/wbfm_exp.py --multi --rounds 4 --k 10 $AB > "$OUT/wbfm_ab.txt" 2>&1 || { tail -5 "$OUT/wbfm_ab.txt"; exit 1; }
  tail -$(( $(echo $AB | wc -w) + 1 )) "$OUT/wbfm_ab.txt"
fi
