#!/bin/bash
# Build an experiment variant of the library: scripts/build_exp.sh NAME -DFLAG=... ...
#   -> orion-sdr_amd/exp/NAME/liborion_sdr_amd.so (timed by tools/wbfm_exp.py)
set -e
cd "$(dirname "$0")/../orion-sdr_amd"
name=$1; shift
make -s -j8 BUILD=build/exp_$name LIB=exp/$name/liborion_sdr_amd.so EXTRA="$*"
