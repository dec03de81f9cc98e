#!/bin/bash
# r02y: ablation A/B on the C3 bench: cos/acos/log of the per-source setup
# and census write (ntrig), the census key derivation (nder); 4 waves/SIMD (w4)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02y
mkdir -p $OUT
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base ntrig nder w4 || exit 1
