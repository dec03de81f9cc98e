#!/bin/bash
# FP with batched temperature-search candidates: parity, then A/B timing.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_fp.py > gpurun_out/r02d/pytest.log 2>&1 \
    || { echo "pytest rc=$?"; tail -30 gpurun_out/r02d/pytest.log; exit 1; }
tail -3 gpurun_out/r02d/pytest.log
S=compton2d_amd/sweep
timeout -k 10 400 python -u tools/fp_ab.py $S/libc2d_w8.so $S/libc2d_w8np.so $S/libc2d_w4.so \
    $S/libc2d_w8n6.so $S/libc2d_w8p.so > gpurun_out/r02d/fp_ab.jsonl 2> gpurun_out/r02d/fp_ab.err \
    || { echo "fp_ab rc=$?"; tail gpurun_out/r02d/fp_ab.err; exit 1; }
cut -c1-330 gpurun_out/r02d/fp_ab.jsonl
