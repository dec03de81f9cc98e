#!/bin/bash
# r02v: Philox cost A/B on the C3 bench: v_mad_u64_u32 products (bit-identical
# streams) and a 7-round ablation (not a product option: measures the RNG share)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02v
mkdir -p $OUT
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base mad p7 || exit 1
