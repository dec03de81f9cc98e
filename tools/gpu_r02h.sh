#!/bin/bash
# Full GPU suite + C3 bench (default flags).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/r02h/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|error" gpurun_out/r02h/pytest.log | head -20; tail -30 gpurun_out/r02h/pytest.log; exit 1; }
tail -3 gpurun_out/r02h/pytest.log
timeout -k 10 600 python -u bench.py > gpurun_out/r02h/bench.json 2> gpurun_out/r02h/bench.err \
    || { echo "bench rc=$?"; tail -20 gpurun_out/r02h/bench.err; exit 1; }
cat gpurun_out/r02h/bench.json
