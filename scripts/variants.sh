#!/bin/bash
# Parity and timing of library variants (orion-sdr_amd/exp/<name>/): for each name in
# V, the GPU tests matching K (parity lines) and the CFG bench line, with
# ORION_SDR_LIB pointing at the variant ("default" = the in-tree library).
#   V="default old lp1" K="lp_dc" CFG=c5 TAG=x bash scripts/variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-var}; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in ${V:-default}; do
  if [ "$v" = default ]; then unset ORION_SDR_LIB; else export ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/$v/liborion_sdr_amd.so; fi
  if [ -n "${K:-}" ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "$K" > "$OUT/tests_$v.log" 2>&1
    rc=$?; [ $rc -le 1 ] || { echo "$v tests rc=$rc"; tail -5 "$OUT/tests_$v.log"; exit $rc; }
    echo "== $v"; grep -E "\[parity\] .*nrmse|passed|failed" "$OUT/tests_$v.log" | grep -v floor | tail -${NL:-12}
  fi
  if [ -n "${CFG:-}" ]; then
    for rep in 1 2; do
      timeout -k 10 180 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu > "$OUT/bench_${v}_$rep.json" 2>&1 || { echo "$v bench failed"; tail -3 "$OUT/bench_${v}_$rep.json"; exit 1; }
      python3 -c "import json;d=json.loads([l for l in open('$OUT/bench_${v}_$rep.json') if 'metric' in l][0]);print('$v', '$CFG', 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
    done
  fi
done
