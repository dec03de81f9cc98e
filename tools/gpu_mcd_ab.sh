#!/bin/bash
# On the GPU box: McDonald series parity + latency probe and the FP bench, default library vs a sweep variant.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/mcd
timeout -k 10 300 python -u -m pytest tests/test_gpu_mcdonald.py tests/test_gpu_fp.py tests/test_gpu_vem.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mcd/tests.log 2>&1 || { tail -20 gpurun_out/mcd/tests.log; exit 1; }
tail -1 gpurun_out/mcd/tests.log
for tag in base "$@"; do
  if [ "$tag" = base ]; then lib=""; else lib=$PWD/compton2d_amd/sweep/$tag/libcompton2d.so; fi
  echo "== $tag"
  C2D_LIBRARY=$lib timeout -k 10 120 python tools/mcd_probe.py
  C2D_LIBRARY=$lib timeout -k 10 300 python tools/fp_bench.py --cpu-zones 2 > gpurun_out/mcd/fp_$tag.json 2> gpurun_out/mcd/fp_$tag.err
  tail -c 600 gpurun_out/mcd/fp_$tag.json
done
