#!/bin/bash
# r02k: transport section timers (C2D_TR_PROF build) on C3
set -o pipefail
mkdir -p gpurun_out/r02k
C2D_LIBRARY=compton2d_amd/sweep/prof/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 7 > gpurun_out/r02k/tr_prof.jsonl 2> gpurun_out/r02k/tr_prof.err
