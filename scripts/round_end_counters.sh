# Round-end evidence, second half (after scripts/round_end.sh): HBM traffic per config
# (FETCH_SIZE / WRITE_SIZE passes), the C2 SQ counters, the reference's six analog round
# trips and the retune cost. Each GPU step under its own limit.
#   TAG=r5f bash scripts/round_end_counters.sh
set -u
OUT=gpurun_out/${TAG:-counters}; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-counters}_traffic CFGS="${TCFGS:-c1 c2 c3 c4 c5}" bash scripts/traffic_session.sh || exit $?
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_LDS" TAG=${TAG:-counters}_pmc bash scripts/pmc_session.sh || exit $?
timeout -k 10 400 python -u tools/roundtrip_bench.py > $OUT/roundtrips.jsonl 2> $OUT/roundtrips.err || { tail -5 $OUT/roundtrips.err; exit 1; }
cat $OUT/roundtrips.jsonl | cut -c1-200
timeout -k 10 300 python -u tools/retune_bench.py > $OUT/retune.jsonl 2> $OUT/retune.err || { tail -5 $OUT/retune.err; exit 1; }
cat $OUT/retune.jsonl
