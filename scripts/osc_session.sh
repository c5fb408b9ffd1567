#!/bin/bash
# Oscillator-consumer session: the GPU tests that touch an oscillator, the per-block
# and modulator lines, and the modulator lines of the experiment builds named in EXP.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-osc}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-osc or rot or nco or mod or ssb or am_ or fm or pm or cw}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|Error" "$OUT/tests.log" | tail -5; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
fi
if [ "${BLOCKS:-1}" = 1 ]; then
timeout -k 10 300 python tools/block_bench.py > "$OUT/blocks.jsonl" 2>&1 || { tail -3 "$OUT/blocks.jsonl"; exit 1; }
grep -o '"row": "[a-z0-9]*", "block": "[^"]*", "n": [0-9]*, "ms_per_call": [0-9.]*' "$OUT/blocks.jsonl"
fi
timeout -k 10 300 python tools/mod_bench.py > "$OUT/mod.jsonl" 2>&1 || { tail -3 "$OUT/mod.jsonl"; exit 1; }
grep -o '"case": "[^"]*", "n": [0-9]*, "ms_per_call": [0-9.]*' "$OUT/mod.jsonl"
for e in ${EXP:-}; do
  ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/$e/liborion_sdr_amd.so timeout -k 10 300 python tools/mod_bench.py > "$OUT/mod_$e.jsonl" 2>&1 || { tail -3 "$OUT/mod_$e.jsonl"; exit 1; }
  echo "== $e"; grep -o '"case": "[^"]*", "n": [0-9]*, "ms_per_call": [0-9.]*' "$OUT/mod_$e.jsonl"
done
