#!/bin/bash
# FP kernel with McDonald producer waves: parity first (short limits), then C3 timing.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02b
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_fp.py tests/test_gpu_c3.py > gpurun_out/r02b/pytest.log 2>&1 \
    || { echo "pytest rc=$?"; tail -30 gpurun_out/r02b/pytest.log; exit 1; }
tail -4 gpurun_out/r02b/pytest.log
timeout -k 10 200 python -u tools/c3_bench.py --sources 10000000 --steps 6 \
    > gpurun_out/r02b/c3_probe.jsonl 2> gpurun_out/r02b/c3_probe.err || { echo "probe rc=$?"; tail gpurun_out/r02b/c3_probe.err; exit 1; }
cut -c1-400 gpurun_out/r02b/c3_probe.jsonl | tail -3
