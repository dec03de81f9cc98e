#!/bin/bash
# kernel-trace stats of the bench with the CDF guide rows off / on (source kernel A/B)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp; cd /tmp
for v in 1 0; do
  C2D_CDF_GUIDE_OFF=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_off$v -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp-offclamp > $O/kt_off$v.json 2> $O/kt_off$v.err || exit 1
  grep -h "source_kernel\|cdf_guide\|bundle_kernel" $O/kt_off$v/run_kernel_stats.csv | cut -d, -f1-5
done
