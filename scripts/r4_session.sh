#!/bin/bash
# Round-4 GPU session: the changed tests, smoke, the driver's C2 command (+ host_fed),
# its rocprof kernel stats, per-block lines, and A/B timings of the round's variants.
# The first crash/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-rotator or nco or dc_pole or contention or host_path or multi_round or mod or ssb}" > "$OUT/tests.log" 2>&1
  rc=$?; grep -E "^\[parity\]|passed|failed|Error" "$OUT/tests.log" | tail -60; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -5 "$OUT/bench_c2.err"; exit 1; }
cut -c1-600 "$OUT/bench_c2.json"; grep -o '"host_fed".*' "$OUT/bench_c2.json" | cut -c1-400
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c2 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-h2d > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
python3 scripts/prof_summary.py "$OUT/prof" | grep -E "avg|k_wbfm" | head -5
timeout -k 10 300 python tools/block_bench.py > "$OUT/blocks.jsonl" 2>&1 || { tail -3 "$OUT/blocks.jsonl"; exit 1; }
cut -c1-200 "$OUT/blocks.jsonl"
if [ "${AB:-1}" = 1 ]; then
  timeout -k 10 300 python tools/wbfm_exp.py --multi --rounds 3 --k 10 base base@3072 base@4096 base@6144 > "$OUT/seg_ab.txt" 2>&1 || { tail -5 "$OUT/seg_ab.txt"; exit 1; }
  tail -5 "$OUT/seg_ab.txt"
fi
if [ "${VAR:-1}" = 1 ]; then
  for v in sc16 rot8; do
    ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/$v/liborion_sdr_amd.so timeout -k 10 300 python tools/block_bench.py --cpu-n 65536 > "$OUT/blocks_$v.jsonl" 2>&1 || { tail -3 "$OUT/blocks_$v.jsonl"; exit 1; }
  done
  ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/firsplit/liborion_sdr_amd.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "fir_lowpass_iq or tx_lowpass" > "$OUT/tests_firsplit.log" 2>&1
  rc=$?; grep -E "firiq|passed|failed" "$OUT/tests_firsplit.log" | tail -8; [ $rc -le 1 ] || exit $rc
  for v in default firsplit; do
    if [ $v = default ]; then unset ORION_SDR_LIB; else export ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/$v/liborion_sdr_amd.so; fi
    for rep in 1 2; do
      timeout -k 10 200 python bench.py --config c1 --steps 30 --warmup 5 --no-cpu > "$OUT/c1_${v}_$rep.json" 2>&1 || { tail -3 "$OUT/c1_${v}_$rep.json"; exit 1; }
      python3 -c "import json;d=json.loads([l for l in open('$OUT/c1_${v}_$rep.json') if 'metric' in l][0]);print('$v c1 ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
    done
  done
  unset ORION_SDR_LIB
  ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/firsplit/liborion_sdr_amd.so timeout -k 10 300 python tools/block_bench.py --cpu-n 65536 > "$OUT/blocks_firsplit.jsonl" 2>&1 || { tail -3 "$OUT/blocks_firsplit.jsonl"; exit 1; }
  for v in default sc16; do
    if [ $v = default ]; then unset ORION_SDR_LIB; else export ORION_SDR_LIB=$PWD/orion-sdr_amd/exp/$v/liborion_sdr_amd.so; fi
    timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu > "$OUT/c5_$v.json" 2>&1 || { tail -3 "$OUT/c5_$v.json"; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$OUT/c5_$v.json') if 'metric' in l][0]);print('$v c5 ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
  done
  unset ORION_SDR_LIB
fi
