#!/bin/bash
# On the GPU box: kernel trace + PMC passes of the C5 light-curve workload (last step).
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_c5
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$ROOT/tools/c5_bench.py --steps 1 --warmup 4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 $B > "$OUT/kt.json" 2> "$OUT/kt.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- python3 $B > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- python3 $B > "$OUT/write.json" 2> "$OUT/write.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM \
    --kernel-trace -d "$OUT/sq" -o run --output-format csv -- python3 $B > "$OUT/sq.json" 2> "$OUT/sq.err"
echo done
