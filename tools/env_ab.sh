#!/bin/bash
# C3 bench A/B of an environment knob, alternating:  bash tools/env_ab.sh <tag> VAR v1 v2 [reps]
set -o pipefail
O=gpurun_out/$1; V=$2; A=$3; B=$4; R=${5:-2}; mkdir -p $O
for r in $(seq $R); do
  for v in $A $B; do
    t=${v//\//_}
    env $V=$v timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp-offclamp \
      > $O/c3_${t}_$r.json 2> $O/c3_${t}_$r.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ps=d['config']['per_step']
print(sys.argv[2], '%.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'g0 %.2f' % ps['transport_gen0_ms'], 'frac %.3f' % d['roofline']['frac'], 'Te %.3f' % ps['mean_Te'], 'cens %.6g' % d['config']['census']['records_at_end'])" $O/c3_${t}_$r.json "$V=$v"
  done
done
