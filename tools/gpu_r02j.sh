#!/bin/bash
# Driver-shaped bench runs: C3 at the round-end arguments, and C4 per GPU.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r02j
true \
    || true

timeout -k 10 600 python -u bench.py --workload c4 --steps 8 --warmup 3 > gpurun_out/r02j/bench_c4_20_5.json 2> gpurun_out/r02j/c4.err \
    || { echo "c4 rc=$?"; tail -20 gpurun_out/r02j/c4.err; exit 1; }
cut -c1-600 gpurun_out/r02j/bench_c4_20_5.json
