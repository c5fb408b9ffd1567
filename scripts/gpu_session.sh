#!/bin/bash
# One GPU session on the gpurun box. Each GPU step has its own time limit; a
# test failure (pytest rc 1) does not stop the session, but any crash, abort,
# fault or timeout does (rc >= 2 from pytest, or any rc != 0 from the others).
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
for s in ${STEPS:-tests smoke bench prof}; do
  case $s in
    tests) step tests 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout=600 -rf; rc=$?
           [ $rc -le 1 ] || exit $rc ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 600 python bench.py --steps ${BSTEPS:-10} --warmup 3 ${BARGS:-} || exit $? ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu ${BARGS:-} || exit $?
           find "$OUT/prof" -name "*kernel_stats*" -exec cat {} \; | head -20 ;;
    pmc)   step pmc 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc1" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BARGS:-} || exit $?
           step pmc2 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc2" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BARGS:-} || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== session done"
