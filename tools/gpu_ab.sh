#!/bin/bash
# On the GPU box: C5 and C2 throughput for the default library and sweep variants.
#   bash tools/gpu_ab.sh base <tag> ...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for tag in "$@"; do
  if [ "$tag" = base ]; then lib=""; else lib=$PWD/compton2d_amd/sweep/$tag/libcompton2d.so; fi
  C2D_LIBRARY=$lib timeout -k 10 200 python tools/c5_bench.py --steps 2 --warmup 3 > gpurun_out/ab/c5_$tag.json 2> gpurun_out/ab/c5_$tag.err
  python -c "import json; d=json.load(open('gpurun_out/ab/c5_$tag.json')); print('c5 $tag', '%.3e'%d['packet_steps_per_s'])"
  C2D_LIBRARY=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/c2_$tag.json 2> gpurun_out/ab/c2_$tag.err
  python -c "import json; d=json.load(open('gpurun_out/ab/c2_$tag.json')); print('c2 $tag', '%.3e'%d['value'], d['roofline']['kernel_ms_avg'])"
done
