#!/bin/bash
# On the GPU box: bench each tuning variant (built by tools/build_sweep.sh).
# Stops at the first failing step.
set -e -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
STEPS=${STEPS:-3}
for tag in "$@"; do
  if [ "$tag" = base ]; then lib=""; else lib=$PWD/compton2d_amd/sweep/$tag/libcompton2d.so; fi
  echo "== $tag $(date +%T)"
  C2D_LIBRARY=$lib timeout -k 10 400 python bench.py --steps $STEPS --warmup 1 --no-cpu-baseline \
      > gpurun_out/sweep/bench_$tag.json 2> gpurun_out/sweep/bench_$tag.err
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep/bench_$tag.json')); print('$tag', '%.3e'%d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['config']['aborted_packets'])"
done
