#!/bin/bash
# On the GPU box: C3 bench (transport-dominated) for sweep variants built by
# tools/build_sweep.sh; prints packet-steps/s and the generation-0 kernel rate.
#   bash tools/gpu_tr_ab.sh base <tag> ...      (STEPS, WARMUP, OUT env)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/tr_ab}
mkdir -p "$OUT"
STEPS=${STEPS:-3}; WARMUP=${WARMUP:-2}
for tag in "$@"; do
  # base: the in-tree library; nb / nrn: it with C2D_BUNDLE=0 / C2D_RN_LDS=0
  envs=""
  case "$tag" in
    base) lib="" ;;
    nb) lib=""; envs="C2D_BUNDLE=0" ;;
    nrn) lib=""; envs="C2D_RN_LDS=0" ;;
    *) lib=$PWD/compton2d_amd/sweep/$tag/libcompton2d.so ;;
  esac
  env $envs C2D_LIBRARY=$lib timeout -k 10 300 python bench.py --steps $STEPS --warmup $WARMUP --no-cpu-baseline \
      > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { echo "$tag failed rc=$?"; tail -5 "$OUT/bench_$tag.err"; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$tag.json')); k=d['kernels']['transport_gen0']
print('%-10s value %.4e  ms/step %.1f  gen0 %.2f ms  gen0 rate %.4e/s  fp %.2f ms' % ('$tag', d['value'], d['ms_per_step'], k['ms_avg'], k['packet_steps_per_launch']/k['ms_avg']*1e3, d['kernels']['fp']['ms_avg']))"
done
