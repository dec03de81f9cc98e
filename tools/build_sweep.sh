#!/bin/bash
# Build tuning variants of libcompton2d.so into compton2d_amd/sweep/<tag>/
# (select one at run time with C2D_LIBRARY=...).
# Usage: tools/build_sweep.sh tag:WPE:CONTRACT[:FLAG,FLAG...[:TRBLOCK[:EXTRA,EXTRA...]]] ...
# (FLAG: fast transport build only; EXTRA: every object)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  IFS=: read -r tag wpe con flags trb extra <<< "$spec"
  out=$ROOT/compton2d_amd/sweep/$tag
  mkdir -p "$out"
  make -s -C "$ROOT/compton2d_amd/csrc" OUT="$out/libcompton2d.so" BUILD="$ROOT/build/sweep/$tag" \
       WPE="$wpe" FAST_CONTRACT="$con" FAST_FLAGS="${flags//,/ }" TRBLOCK="${trb:-256}" EXTRA="${extra//,/ }" -j4
done
