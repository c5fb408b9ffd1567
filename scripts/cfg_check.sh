#!/bin/bash
# GPU iteration on one config: the GPU tests matching K, the config's bench under
# rocprofv3 kernel trace (per-kernel averages), then its bench line.
#   K="lpdc or ssb" CFG=c5 TAG=x bash scripts/cfg_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-cfg}; mkdir -p "$OUT"; export TMPDIR=/tmp
CFG=${CFG:-c2}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-wbfm}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "parity|passed|failed|Error|error" "$OUT/tests.log" | tail -${NT:-30}
[ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 scripts/prof_summary.py "$OUT/prof" | grep avg | tee "$OUT/kstats.txt"; rm -rf "$OUT/prof"
timeout -k 10 180 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu 2>&1 | grep metric | tee "$OUT/bench.json" | cut -c1-300
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('frac',d['roofline']['frac'],'ms',d['ms_per_step'])"
