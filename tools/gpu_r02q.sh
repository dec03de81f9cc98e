#!/bin/bash
# r02q: bundle-kernel occupancy / block-size / contraction A/B on C3, then
# the section timers of the bundle kernel (prof build)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02q
mkdir -p $OUT
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base w2 w3b256 w4b256 w4fma || exit 1
C2D_LIBRARY=$PWD/compton2d_amd/sweep/prof/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 6 > $OUT/tr_prof.jsonl 2> $OUT/tr_prof.err \
  || { echo "tr_prof rc=$?"; tail -5 $OUT/tr_prof.err; exit 1; }
tail -1 $OUT/tr_prof.jsonl
