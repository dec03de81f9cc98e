#!/bin/bash
# C3 bench A/B/... of library builds, alternating:  bash tools/lib_ab.sh <tag> <reps> lib1 lib2 ...
# (builds from tools/build_sweep.sh; the timed steps only, no CPU baseline / off-clamp FP)
set -o pipefail
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq $R); do
  for v in "$@"; do
    t=${v//\//_}
    C2D_LIBRARY=$v timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp-offclamp \
      > $O/c3_${t}_$r.json 2> $O/c3_${t}_$r.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ps=d['config']['per_step']
print(sys.argv[2], '%.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'g0 %.2f' % ps['transport_gen0_ms'], 'frac %.3f' % d['roofline']['frac'], 'Te %.3f' % ps['mean_Te'], 'cens %.6g' % d['config']['census']['records_at_end'])" $O/c3_${t}_$r.json "$v"
  done
done
