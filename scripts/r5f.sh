# Round-5 evidence, second half: HBM traffic per config, the C2 SQ counters, the
# reference's six analog round trips. Each GPU step under its own limit.
set -u
OUT=gpurun_out/${TAG:-r5f}; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r5f}_traffic CFGS="${TCFGS:-c1 c2 c3 c4 c5}" bash scripts/traffic_session.sh || exit $?
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_LDS" TAG=${TAG:-r5f}_pmc bash scripts/pmc_session.sh || exit $?
timeout -k 10 400 python -u tools/roundtrip_bench.py > $OUT/roundtrips.jsonl 2> $OUT/roundtrips.err || { tail -5 $OUT/roundtrips.err; exit 1; }
cat $OUT/roundtrips.jsonl | cut -c1-200
