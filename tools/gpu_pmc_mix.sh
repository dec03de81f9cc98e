#!/bin/bash
# On the GPU box: instruction-mix PMC passes of the transport kernel
# (each pass its own run, --kernel-trace only).  Lists the available SQ
# counters first so the pass contents can be checked.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/mix
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
B="$ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1"
pass() {
  local tag=$1; shift
  echo "== $tag $(date +%T)"
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$tag" -o run --output-format csv -- \
      python3 $B > "$OUT/bench_$tag.json" 2> "$OUT/$tag.err"
}
pass f64 SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT
pass busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES
echo "== done $(date +%T)"
