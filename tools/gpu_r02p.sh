#!/bin/bash
# r02p: HEAD re-verification after the container restore: full GPU suite,
# driver-shaped C3 bench (20 timed + 5 warm-up, with cpu_baseline), then the
# kernel-trace + PMC passes (tools/gpu_profile.sh).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02p
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest.txt 2>&1
rc=$?
tail -8 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
bash tools/gpu_profile.sh r02p
