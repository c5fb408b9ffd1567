#!/bin/bash
# Build the library as of a git revision (default HEAD) into orion-sdr_amd/exp/NAME/,
# for paired in-process A/B against the working tree (tools/wbfm_exp.py --multi):
#   scripts/build_variant.sh NAME [REV]
# A variant is a source snapshot built out of tree; it never writes lib/.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; rev=${2:-HEAD}
src=/tmp/orion_variant_$name
rm -rf "$src"; mkdir -p "$src"
git -C "$ROOT" archive "$rev" orion-sdr_amd/csrc orion-sdr_amd/Makefile include | tar -x -C "$src"
make -s -C "$src/orion-sdr_amd" -j8 LIB="$ROOT/orion-sdr_amd/exp/$name/liborion_sdr_amd.so"
