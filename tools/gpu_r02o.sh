#!/bin/bash
# r02o: full GPU suite with the bundle kernel + census chunks, then C3 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/r02o/pytest.txt 2>&1
rc=$?
tail -15 gpurun_out/r02o/pytest.txt
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r02o bash tools/gpu_tr_ab.sh base nb
