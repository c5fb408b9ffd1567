#!/bin/bash
# k_scan_sp change check: scan-path GPU parity, then the per-block bench with the
# single pass and with ORION_SCAN_3K=1 (three-kernel scan).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-scansp}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-single_pass or lp_cascade or fm_demod or pm_ssb or ssb_phasing or chain or mod}" > "$OUT/tests.log" 2>&1
rc=$?; grep -E "single-pass|passed|failed|Error" "$OUT/tests.log" | tail -40; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/block_bench.py --cpu-n 65536 > "$OUT/sp.jsonl" 2>&1 || { tail -5 "$OUT/sp.jsonl"; exit 1; }
ORION_SCAN_FULL=1 timeout -k 10 300 python tools/block_bench.py --cpu-n 65536 > "$OUT/full.jsonl" 2>&1 || { tail -5 "$OUT/full.jsonl"; exit 1; }
python3 - "$OUT" <<'PY'
import json,sys
a=[json.loads(l) for l in open(sys.argv[1]+'/sp.jsonl') if l.startswith('{')]
b=[json.loads(l) for l in open(sys.argv[1]+'/full.jsonl') if l.startswith('{')]
for x,y in zip(a,b): print(f"{x['block'][:45]:45s} single {x['ms_per_call']:.4f} ms ({x['frac_of_8TBs']:.3f})  full {y['ms_per_call']:.4f} ms ({y['frac_of_8TBs']:.3f})")
PY
