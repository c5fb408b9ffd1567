#!/bin/bash
# PMC passes of tools/wbfm_exp.py --child on library variants (one rocprofv3 run per
# variant and counter set, each under its own time limit).
#   VARS="base l2front" SETS="A B;C D" TAG=x bash scripts/pmc_var.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmcvar}; mkdir -p "$OUT"; export TMPDIR=/tmp
IFS=';' read -ra SS <<< "$SETS"
for v in $VARS; do
  i=0; mkdir -p "$OUT/$v"
  for set in "${SS[@]}"; do
    i=$((i+1))
    if [ "$v" = base ]; then lib=orion-sdr_amd/lib/liborion_sdr_amd.so; else lib=orion-sdr_amd/exp/$v/liborion_sdr_amd.so; fi
    ORION_SDR_LIB=$PWD/$lib timeout -k 10 90 rocprofv3 --pmc $set -d "$OUT/$v/p$i" -o run -- python3 tools/wbfm_exp.py --child --k 3 --w 1 > "$OUT/$v/p$i.log" 2>&1 || { echo "$v pass $i failed"; tail -5 "$OUT/$v/p$i.log"; exit 1; }
  done
  echo "== $v"; python3 scripts/prof_summary.py "$OUT/$v" | tee "$OUT/$v/summary.txt"
done
