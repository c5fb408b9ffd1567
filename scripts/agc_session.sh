mkdir -p gpurun_out/agc2 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "agc or overlap" > gpurun_out/agc2/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error" gpurun_out/agc2/tests.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/agc_bench.py > gpurun_out/agc2/bench.jsonl 2>&1 || exit 1
cat gpurun_out/agc2/bench.jsonl
ORION_AGC_SEQ_DIV=100000000 timeout -k 10 200 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import agc_bench as a
a.run(True, 10e6, 0.2, 5.0, 0.5, 1<<24, reps=2)
a.run(True, 48e3, 1.0, 500.0, 0.3, 1<<24, reps=2)
a.run(True, 48e3, 1.0, 20.0, 0.3, 1<<24, reps=2)
" 2>&1 | grep case
