#!/bin/bash
# C4 per GPU (bench --workload c4, 8 timed + 3 warm-up) and the C5 EC
# light-curve tool on the current kernels.   TAG=<tag> bash tools/gpu_c4c5.sh
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-c4c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --workload c4 --steps 8 --warmup 3 --no-cpu-baseline \
    > $OUT/bench_c4_8_3.json 2> $OUT/c4.err || { echo "c4 rc=$?"; tail -20 $OUT/c4.err; exit 1; }
cut -c1-200 $OUT/bench_c4_8_3.json
timeout -k 10 400 python -u tools/c5_bench.py > $OUT/c5_bench.json 2> $OUT/c5.err \
    || { echo "c5 rc=$?"; tail -20 $OUT/c5.err; exit 1; }
tail -c 600 $OUT/c5_bench.json
