#!/bin/bash
# Round-6 check session: full GPU suite, then the default C2 line, C5 at the default
# command, C5F, and the two-rank rehearsal on one device (gloo, shared device 0,
# stream shards gathered and compared with one call). The first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6s}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -2 "$OUT/tests.log"; grep -E "^\.*\[parity\]|passed|failed" "$OUT/tests.log" | sed 's/^\.*//' > "$OUT/parity.txt"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -5 "$OUT/bench_c2.err"; exit 1; }
cut -c1-400 "$OUT/bench_c2.json"
for c in ${CFGS:-c5 c5f}; do
  timeout -k 10 300 python bench.py --config $c > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -5 "$OUT/bench_$c.err"; exit 1; }
  cut -c1-300 "$OUT/bench_$c.json"
done
if [ "${DIST:-1}" = 1 ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --samples 4194304 --steps 10 --warmup 2 --dist-backend gloo --device-map 0,0 --check-shards --no-cpu \
    > "$OUT/bench_dist2.json" 2> "$OUT/bench_dist2.err" || { tail -8 "$OUT/bench_dist2.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_dist2.json').read().strip().splitlines()[-1]); print('dist2', d['n_gpus'], d['value'], d['shard_check'])"
fi
