#!/bin/bash
# fast-FP off-clamp A/B of builds (compton2d_amd/sweep/<t>, "base" = in-tree),
# gamma_bar memo emptied before every update (C2D_FPF_MEMO_RESET=1):
#   bash tools/fp_ab.sh <tag> <build> [build ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for t in "$@"; do
  lib=$PWD/compton2d_amd/libcompton2d.so; [ "$t" = base ] || lib=$PWD/compton2d_amd/sweep/$t/libcompton2d.so
  C2D_FPF_MEMO_RESET=1 C2D_LIBRARY=$lib timeout -k 10 300 python tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 \
    --cpu-zones 8 --mode fast > $O/fp_$t.out 2> $O/fp_$t.err || exit 1
  echo "$t: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.2f ms (first call %.2f), f_nt dev %.1e, Te equal %s' % (d['kernel_ms'], d['kernel_ms_first_call'], d['f_nt_max_dev_vs_oracle_on_sample'], d['Te_new_equal_on_sample']))" $O/fp_$t.out)"
done
