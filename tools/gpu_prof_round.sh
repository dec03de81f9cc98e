#!/bin/bash
# Section timers (C2D_TR_PROF build in compton2d_amd/sweep/prof) and the PMC
# passes of the C3 bench:  TAG=<name> bash tools/gpu_prof_round.sh
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-cur}
mkdir -p gpurun_out/$TAG
C2D_LIBRARY=$PWD/compton2d_amd/sweep/prof/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 4 > gpurun_out/$TAG/tr_prof.jsonl 2> gpurun_out/$TAG/tr_prof.err \
  || { echo "tr_prof rc=$?"; tail -5 gpurun_out/$TAG/tr_prof.err; exit 1; }
tail -1 gpurun_out/$TAG/tr_prof.jsonl
bash tools/gpu_profile.sh $TAG
