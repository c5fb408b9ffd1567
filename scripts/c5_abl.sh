set -u
for v in base sp2 sp4 sp6 base; do
  if [ $v = base ]; then L=""; else L="ORION_SDR_LIB=$PWD/orion-sdr_amd/lib/abl/liborion_$v.so"; fi
  env $L timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --config c5 2>&1 | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
