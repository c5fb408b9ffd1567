#!/bin/bash
# Multi-rank rehearsal of bench.py on ONE GPU (the driver's N > 1 command shape, ranks
# sharing device 0 over gloo): NPROC ranks, C2 cut in time (stream shards, --check-shards
# gathers every rank's audio and compares it with one call over the whole stream), then
# the C4 / C5 channel ranges. RCCL wants one rank per GPU, so the backend is gloo here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dist}; mkdir -p "$OUT"; export TMPDIR=/tmp
N=${NPROC:-4}; MAP=$(python3 -c "print(','.join(['0'] * $N))")
for c in ${CFGS:-c2 c4 c5}; do
  extra=""; [ "$c" = c2 ] && extra="--check-shards --samples 4194304"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + RANDOM % 300)) bench.py --config $c --gpus $N --steps 5 --warmup 2 --dist-backend gloo \
    --device-map $MAP --no-cpu $extra > "$OUT/bench_${c}_n$N.json" 2> "$OUT/bench_${c}_n$N.err" \
    || { tail -8 "$OUT/bench_${c}_n$N.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_${c}_n$N.json').read().strip().splitlines()[-1]); print('$c', d['n_gpus'], d['value'], d['config'].get('parallelism'), d.get('shard_check'))"
done
