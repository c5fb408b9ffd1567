#!/bin/bash
# Ad-hoc timing experiments on the GPU box: each case runs bench.py under
# rocprofv3 --kernel-trace with the given environment and prints the per-kernel
# average duration (databases are summarised on the box and deleted).
#   CASES="tag:VAR=v,VAR=v tag2:..."  bash scripts/exp_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-exp}; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in $CASES; do
  tag=${c%%:*}; envs=${c#*:}
  env ${envs//,/ } timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu ${BARGS:-} > "$OUT/$tag.log" 2>&1 || { echo "FAIL $tag"; tail -5 "$OUT/$tag.log"; exit 1; }
  python3 scripts/prof_summary.py "$OUT/$tag" | grep avg | sed "s/^/$tag /" | tee -a "$OUT/summary.txt"; rm -rf "$OUT/$tag"
done
