#!/bin/bash
# On the GPU box: L2 (TCC) and vector L1 (TCP) hit counters of the bench
# workload's generation-0 launches, one rocprofv3 --pmc pass
# (MI355X_MICROARCH.md: counters in their own pass, kernel trace only).
#   tools/gpu_cache_pmc.sh <tag> [bench args...]   (gpurun_out/prof_<tag>/cache)
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-cur}
shift || true
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$ROOT/bench.py --no-cpu-baseline --no-fp-offclamp $*"
# PMC="..." overrides the counter set (at most 4 TCC_ and 4 TCP_ counters per pass)
PMC=${PMC:-TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum}
timeout -k 10 300 rocprofv3 --pmc $PMC \
    --kernel-trace -d "$OUT/cache" -o run --output-format csv -- \
    python3 $B --steps ${STEPS:-3} --warmup ${WARMUP:-1} > "$OUT/bench_cache.json" 2> "$OUT/cache.err"
python3 - "$OUT/cache" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "bundle_kernel" in k or "source_kernel" in k:
        acc[k.split("(")[0][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    print(k, {n: "%.4g" % v for n, v in c.items()}, "L2 hit %.3f" % (h / max(h + m, 1)))
PY
