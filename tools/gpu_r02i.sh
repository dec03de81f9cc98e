#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02i
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu -s \
    tests/test_gpu_spectrum.py > gpurun_out/r02i/pytest_spectrum.log 2>&1 \
    || { echo "pytest rc=$?"; tail -30 gpurun_out/r02i/pytest_spectrum.log; exit 1; }
grep -E "rel L2|passed" gpurun_out/r02i/pytest_spectrum.log
bash tools/gpu_profile.sh r02i
