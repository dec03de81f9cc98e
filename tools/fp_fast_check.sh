#!/bin/bash
# C2D_FP_FAST check on the GPU box: the fast-FP parity tests, the off-clamp
# FP bench (30x9, varied zones) and its section timers, for the in-tree
# library and each sweep build named after the tag (compton2d_amd/sweep/<t>,
# profile builds sweep/<t>prof and sweep/<t>sec, or fpprof and fpsec for the
# in-tree one).
#   bash tools/fp_fast_check.sh <tag> [sweep ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp.py tests/test_gpu_c3.py -k "fast" -x -q --timeout 200 > $O/pytest_fast.out 2>&1 || { tail -30 $O/pytest_fast.out; exit 1; }
tail -1 $O/pytest_fast.out
for t in base "$@"; do
  lib=""; prof=$PWD/compton2d_amd/sweep/fpprof/libcompton2d.so
  if [ "$t" != base ]; then lib=$PWD/compton2d_amd/sweep/$t/libcompton2d.so; prof=$PWD/compton2d_amd/sweep/${t}prof/libcompton2d.so; fi
  C2D_LIBRARY=$lib timeout -k 10 300 python tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 --cpu-zones 8 --mode fast > $O/fp_fast_$t.out 2> $O/fp_fast_$t.err || exit 1
  echo "$t: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.2f ms (first call %.2f), f_nt dev %.1e, Te equal %s' % (d['kernel_ms'], d['kernel_ms_first_call'], d['f_nt_max_dev_vs_oracle_on_sample'], d['Te_new_equal_on_sample']))" $O/fp_fast_$t.out)"
  if [ -f "$prof" ]; then
    C2D_LIBRARY=$prof timeout -k 10 300 python tools/fp_prof.py --nz 30 --nr 9 --vary --mode fast > $O/fpprof_$t.out 2>&1 || exit 1
    tail -1 $O/fpprof_$t.out
  fi
  sec=$PWD/compton2d_amd/sweep/fpsec/libcompton2d.so
  [ "$t" != base ] && sec=$PWD/compton2d_amd/sweep/${t}sec/libcompton2d.so
  if [ -f "$sec" ]; then
    C2D_LIBRARY=$sec timeout -k 10 300 python tools/fp_prof.py --nz 30 --nr 9 --vary --mode fast --sections > $O/fpsec_$t.out 2>&1 || exit 1
    tail -1 $O/fpsec_$t.out
  fi
  memo=$PWD/compton2d_amd/sweep/fpmemo/libcompton2d.so
  [ "$t" != base ] && memo=$PWD/compton2d_amd/sweep/${t}memo/libcompton2d.so
  if [ -f "$memo" ]; then
    C2D_LIBRARY=$memo timeout -k 10 300 python tools/fp_prof.py --nz 30 --nr 9 --vary --mode fast --memo > $O/fpmemo_$t.out 2>&1 || exit 1
    tail -1 $O/fpmemo_$t.out
  fi
done
