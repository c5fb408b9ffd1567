#!/bin/bash
# Timing-experiment builds of the engine (not the product): $SRC (default k_wbfm).hip compiled
# with extra -D flags, linked with the normal objects into
# orion-sdr_amd/lib/abl/liborion_<tag>.so; select one with ORION_SDR_LIB.
#   bash scripts/build_var.sh "nb:-DORION_SEG_ABL=1" "np:-DORION_SEG_PRIO=0"
set -e
cd "$(dirname "$0")/../orion-sdr_amd"
make -s
src=${SRC:-k_wbfm}
mkdir -p lib/abl build/abl
for v in "$@"; do
  tag=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 $flags \
    -c csrc/$src.hip -o build/abl/${src}_$tag.o &
done
wait
objs=$(ls build/*.o | grep -v "/$src.o")
for v in "$@"; do
  tag=${v%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/abl/liborion_$tag.so build/abl/${src}_$tag.o $objs
done
