#!/bin/bash
# Build the library as of a git revision (default HEAD; "." = the working tree) into
# orion-sdr_amd/exp/NAME/, for paired in-process A/B (tools/ab_variants.py,
# tools/wbfm_exp.py --multi):   scripts/build_variant.sh NAME [REV]
# A variant is a source snapshot built out of tree; it never writes lib/.
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; rev=${2:-HEAD}
src=/tmp/orion_variant_$name
rm -rf "$src"; mkdir -p "$src/orion-sdr_amd"
if [ "$rev" = "." ]; then
  cp -r "$ROOT/orion-sdr_amd/csrc" "$ROOT/orion-sdr_amd/Makefile" "$src/orion-sdr_amd/"; cp -r "$ROOT/include" "$src/"
else
  git -C "$ROOT" archive "$rev" orion-sdr_amd/csrc orion-sdr_amd/Makefile include | tar -x -C "$src"
fi
make -s -C "$src/orion-sdr_amd" -j8 DEFS="${DEFS:-}" LIB="$ROOT/orion-sdr_amd/exp/$name/liborion_sdr_amd.so"
