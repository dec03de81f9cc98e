#!/bin/bash
# On the GPU box: kernel-trace + PMC passes of the bench workload.
#   tools/gpu_profile.sh <tag> [bench args...]   (results under gpurun_out/prof_<tag>/)
# PMC passes run separately (FETCH_SIZE and WRITE_SIZE cannot share a pass),
# each with --kernel-trace only, as MI355X_MICROARCH.md prescribes.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-cur}
shift || true
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$ROOT/bench.py --no-cpu-baseline --no-fp-offclamp $*"
# every pass runs the bench's own configuration (the driver's default K/W)
K=${STEPS:-5}; W=${WARMUP:-2}
echo "== kernel trace $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python3 $B --steps $K --warmup $W > "$OUT/bench_kt.json" 2> "$OUT/kt.err"
echo "== FETCH_SIZE $(date +%T)"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- \
    python3 $B --steps $K --warmup $W > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
echo "== WRITE_SIZE $(date +%T)"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- \
    python3 $B --steps $K --warmup $W > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo "== SQ $(date +%T)"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM \
    --kernel-trace -d "$OUT/sq" -o run --output-format csv -- \
    python3 $B --steps $K --warmup $W > "$OUT/bench_sq.json" 2> "$OUT/sq.err"
echo "== done $(date +%T)"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
