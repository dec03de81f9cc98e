#!/bin/bash
# FP A/B: single-wave series vs producer waves (batch sizes), with section timers.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
S=compton2d_amd/sweep
timeout -k 10 300 python -u tools/fp_ab.py $S/libc2d_w1.so $S/libc2d_w4.so $S/libc2d_w4b8.so \
    $S/libc2d_w4b32.so $S/libc2d_w1p.so $S/libc2d_w4p.so > gpurun_out/r02c/fp_ab.jsonl 2> gpurun_out/r02c/fp_ab.err \
    || { echo "fp_ab rc=$?"; tail gpurun_out/r02c/fp_ab.err; exit 1; }
cat gpurun_out/r02c/fp_ab.jsonl
