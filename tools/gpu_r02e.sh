#!/bin/bash
# FP waves-per-zone A/B (runtime C2D_FP_WAVES) on C3 and the tiled steady case.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02e
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_fp.py > gpurun_out/r02e/pytest.log 2>&1 \
    || { echo "pytest rc=$?"; tail -30 gpurun_out/r02e/pytest.log; exit 1; }
tail -2 gpurun_out/r02e/pytest.log
for w in 1 2 4 8 auto; do
  if [ $w = auto ]; then unset C2D_FP_WAVES; else export C2D_FP_WAVES=$w; fi
  echo "== waves $w"
  timeout -k 10 200 python -u tools/fp_ab.py compton2d_amd/libcompton2d.so > gpurun_out/r02e/fp_ab_$w.jsonl 2> gpurun_out/r02e/fp_ab_$w.err \
      || { echo "fp_ab rc=$?"; tail gpurun_out/r02e/fp_ab_$w.err; exit 1; }
  cut -c1-120 gpurun_out/r02e/fp_ab_$w.jsonl
done
