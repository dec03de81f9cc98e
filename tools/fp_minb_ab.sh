#!/bin/bash
# fast FP at one vs two workgroups per CU (sweep build fpm2: -DC2D_FPF_MINB=2,
# <= 256 VGPRs), on C3's clamped zones (coupled bench, --fp-mode fast) and off
# the clamp (tools/fp_bench.py --vary, memo emptied): bash tools/fp_minb_ab.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
B=$PWD/compton2d_amd/libcompton2d.so; M=$PWD/compton2d_amd/sweep/fpm2/libcompton2d.so
c3() {  # c3 <name> <lib> [env...]
  local n=$1 lib=$2; shift 2
  env C2D_LIBRARY=$lib "$@" timeout -k 10 400 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fp-offclamp \
    --fp-mode fast > $O/c3_$n.json 2> $O/c3_$n.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ps=d['config']['per_step']
print('c3', sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'fp_kernel %.3f' % ps['fp_kernel_ms'], 'Te %.4f' % ps['mean_Te'])" $O/c3_$n.json $n
}
off() {  # off <name> <lib> [env...]
  local n=$1 lib=$2; shift 2
  env C2D_LIBRARY=$lib C2D_FPF_MEMO_RESET=1 "$@" timeout -k 10 300 python tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 \
    --cpu-zones 8 --mode fast > $O/off_$n.out 2> $O/off_$n.err || exit 1
  echo "off $n: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.2f ms (first call %.2f), f_nt dev %.1e, Te equal %s' % (d['kernel_ms'], d['kernel_ms_first_call'], d['f_nt_max_dev_vs_oracle_on_sample'], d['Te_new_equal_on_sample']))" $O/off_$n.out)"
}
c3 base $B
c3 m2_grid0 $M C2D_FPF_GRID=0
c3 m2_grid512 $M C2D_FPF_GRID=512
off base $B
off m2_grid0 $M C2D_FPF_GRID=0
off m2_grid512 $M C2D_FPF_GRID=512
off m2 $M
