#!/bin/bash
# kernel-trace stats of a short bench per build (source-kernel A/B):
#   tools/src_kt.sh <tag> <build> [build ...]   (build: compton2d_amd/sweep/<t>/, "base" = in-tree)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp; cd /tmp
for t in "$@"; do
  lib=$ROOT/compton2d_amd/libcompton2d.so; [ "$t" = base ] || lib=$ROOT/compton2d_amd/sweep/$t/libcompton2d.so
  C2D_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$t -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp-offclamp > $O/kt_$t.json 2> $O/kt_$t.err || exit 1
  echo "== $t"; grep -h "source_kernel\|bundle_kernel" $O/kt_$t/run_kernel_stats.csv | cut -d, -f1-4
done
