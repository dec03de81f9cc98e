#!/bin/bash
# r02w: ablation A/B on the C3 bench: per-probe absorption-point sampling
# (nabs), n_field atomics (nonf) vs the product build
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02w
mkdir -p $OUT
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base nabs || exit 1
