#!/bin/bash
# Round evidence on the GPU box: smoke, driver-shaped C3 bench (20 timed + 5
# warm-up, with cpu_baseline), kernel-trace + PMC passes of the same 20 + 5
# command, pmc_latest.json for bench.py.   TAG=<tag> bash tools/gpu_evidence.sh
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-cur}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_c3_20_5.json 2> $OUT/bench.err \
    || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench_c3_20_5.json
STEPS=20 WARMUP=5 bash tools/gpu_profile.sh $TAG || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_$TAG --latest c3_30x9_100000000_fast \
  "profiles/$TAG/summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ passes of bench.py --steps 20 --warmup 5 on C3, the 20 timed generation-0 dispatches; FETCH_SIZE x2 per MI355X_MICROARCH.md)" > /dev/null
cp profiles/pmc_latest.json $OUT/
