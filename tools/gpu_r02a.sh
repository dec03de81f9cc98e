#!/bin/bash
# Round-2 first GPU pass: new GPU tests, a C3 census-growth probe, the bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_c3.py tests/test_fortran_binding.py tests/test_gpu_parity.py \
    > gpurun_out/r02a/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r02a/pytest.log; exit 1; }
tail -5 gpurun_out/r02a/pytest.log
timeout -k 10 300 python -u tools/c3_bench.py --sources 10000000 --steps 25 \
    > gpurun_out/r02a/c3_probe.jsonl 2> gpurun_out/r02a/c3_probe.err || { echo "probe rc=$?"; tail gpurun_out/r02a/c3_probe.err; exit 1; }
tail -3 gpurun_out/r02a/c3_probe.jsonl
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err || { echo "bench rc=$?"; tail gpurun_out/r02a/bench.err; exit 1; }
cat gpurun_out/r02a/bench.json
