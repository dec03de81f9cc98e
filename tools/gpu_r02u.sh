#!/bin/bash
# r02u: section timers of the bundle kernel (prof build) and the n_field
# ablation A/B on the C3 bench (transport-dominated)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02u
mkdir -p $OUT
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base nonf || exit 1
C2D_LIBRARY=$PWD/compton2d_amd/sweep/prof/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 8 > $OUT/tr_prof.jsonl 2> $OUT/tr_prof.err \
  || { echo "tr_prof rc=$?"; tail -5 $OUT/tr_prof.err; exit 1; }
tail -2 $OUT/tr_prof.jsonl
