#!/bin/bash
# On the GPU box: SQ counters of the source kernel (c2d_source_kernel_fast)
# over a short bench, one rocprofv3 --pmc pass per counter set
# (MI355X_MICROARCH.md: counters in their own pass, kernel trace only).
#   tools/src_pmc.sh <tag> [bench args...]   (gpurun_out/<tag>/src_pmc_*)
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-cur}
shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$ROOT/bench.py --no-cpu-baseline --no-fp-offclamp $*"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex source_kernel --kernel-trace \
      -d "$OUT/src_pmc_$i" -o run --output-format csv -- \
      python3 $B --steps ${STEPS:-2} --warmup ${WARMUP:-1} > "$OUT/src_pmc_$i.json" 2> "$OUT/src_pmc_$i.err"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/src_pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "source_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
n = {k: len(v) for k, v in disp.items()}
w = acc["SQ_WAVES"] / max(n.get("SQ_WAVES", 1), 1)
print("source kernel dispatches", n.get("SQ_WAVES"), "waves/dispatch %.0f" % w)
for k in sorted(acc):
    per = acc[k] / max(n[k], 1)
    print("%-24s per dispatch %.4g  per wave %.1f" % (k, per, per / max(w, 1)))
PY
