#!/bin/bash
# Timing-experiment builds of the engine (not the product): k_wbfm.hip compiled
# with -DORION_FU_ABL=<bits> and linked with the normal objects into
# orion-sdr_amd/lib/abl/liborion_abl<bits>.so; select one with ORION_SDR_LIB.
#   bash scripts/build_abl.sh 2 4 6
set -e
cd "$(dirname "$0")/../orion-sdr_amd"
make -s
mkdir -p lib/abl build/abl
for b in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -DORION_FU_ABL=$b \
    -c csrc/k_wbfm.hip -o build/abl/k_wbfm_$b.o &
done
wait
for b in "$@"; do
  objs=$(ls build/*.o | grep -v k_wbfm.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/abl/liborion_abl$b.so build/abl/k_wbfm_$b.o $objs
done
ls -la lib/abl
