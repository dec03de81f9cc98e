#!/bin/bash
# r02m: bundle kernel — section timers and PMC passes on C3
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02m
C2D_LIBRARY=$PWD/compton2d_amd/sweep/prof/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 4 > gpurun_out/r02m/tr_prof.jsonl 2> gpurun_out/r02m/tr_prof.err \
  || { echo "tr_prof rc=$?"; tail -5 gpurun_out/r02m/tr_prof.err; exit 1; }
cat gpurun_out/r02m/tr_prof.jsonl | tail -1
bash tools/gpu_profile.sh r02m
