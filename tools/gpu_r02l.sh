#!/bin/bash
# r02l: probe bundles — exact-kernel parity vs the oracle, then C3 A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02l
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_census_restart.py tests/test_gpu_sharding.py tests/test_gpu_c3.py \
    > gpurun_out/r02l/pytest.txt 2>&1
rc=$?
tail -15 gpurun_out/r02l/pytest.txt
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r02l bash tools/gpu_tr_ab.sh ${AB:-base nb nrn}
