#!/bin/bash
# On the GPU box: bench the transport with several C2D_REGEN values (and the
# library under compton2d_amd/sweep/old as a reference point).
set -e -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
STEPS=${STEPS:-3}
run() {
  local tag=$1 lib=$2 regen=$3
  C2D_LIBRARY=$lib C2D_REGEN=$regen timeout -k 10 300 python bench.py --steps $STEPS --warmup 1 --no-cpu-baseline \
      > gpurun_out/sweep/bench_$tag.json 2> gpurun_out/sweep/bench_$tag.err
  python -c "import json; d=json.load(open('gpurun_out/sweep/bench_$tag.json')); print('$tag', '%.3e'%d['value'], '%.2f'%d['ms_per_step'], '%.2f'%d['roofline']['kernel_ms_avg'], d['config']['aborted_packets'])"
}
[ -f compton2d_amd/sweep/old/libcompton2d.so ] && run old $PWD/compton2d_amd/sweep/old/libcompton2d.so 16
for r in "$@"; do run regen$r "" $r; done
