#!/bin/bash
# One GPU session on the gpurun box. Each GPU step has its own time limit; a
# test failure (pytest rc 1) does not stop the session, but any crash, abort,
# fault or timeout does (rc >= 2 from pytest, or any rc != 0 from the others).
#   STEPS="tests smoke bench prof pmc"   TAG=<out subdir>   BARGS=<bench args>
#   PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU ..."  (one rocprofv3 run per set)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-s}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== [$name] $(date +%T) $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n ${TAILN:-25} "$OUT/$name.log"
  return $rc
}
DEFAULT_PMC="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY;SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for s in ${STEPS:-tests smoke bench prof}; do
  case $s in
    tests) step tests 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout=600 -rf ${PYARGS:-}; rc=$?
           [ $rc -le 1 ] || exit $rc ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 600 python bench.py --steps ${BSTEPS:-10} --warmup 3 ${BARGS:-} || exit $? ;;
    cfgs)  for c in c3 c4 c5; do  # the other BASELINE configs
             step bench_$c 600 python bench.py --steps 10 --warmup 3 --no-cpu --config $c || exit $?
             step prof_$c 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$c" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --config $c || exit $?
             find "$OUT/prof_$c" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$c.csv" \;
           done ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu ${BARGS:-} || exit $?
           find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; ;;
    pmc)   i=0
           IFS=';' read -ra SETS <<< "${PMC_SETS:-$DEFAULT_PMC}"
           for set in "${SETS[@]}"; do
             i=$((i+1))
             step pmc$i 600 rocprofv3 --pmc $set -f csv -d "$OUT/pmc$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BARGS:-} || exit $?
           done ;;
    list)  step list 120 rocprofv3 -L || exit $? ;;
    abl)   for v in ${ABLS:-0 1 2 4 8 3 14 15 16 32 48}; do  # timing ablations (k_wbfm.hip ABL)
             ORION_WBFM_ABL=$v step abl$v 300 rocprofv3 --kernel-trace --stats -d "$OUT/abl$v" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu ${BARGS:-} || exit $?
             python3 scripts/prof_summary.py "$OUT/abl$v" | sed "s/^/ABL=$v /" | grep avg; rm -rf "$OUT/abl$v"
           done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== session done"
