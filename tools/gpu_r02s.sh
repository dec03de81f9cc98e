#!/bin/bash
# r02s: bucket-table bin lookups, 3 waves/SIMD x 256-thread groups by
# default: GPU suite, C3 bench, section timers
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest.txt 2>&1
rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.txt | head -20; exit $rc; }
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base || exit 1
C2D_FP_MEMO=0 timeout -k 10 300 python bench.py --steps 4 --warmup 4 --no-cpu-baseline > $OUT/bench_nomemo.json 2> $OUT/bench_nomemo.err || exit 1
python -c "import json; d=json.load(open('$OUT/bench_nomemo.json')); print('no memo: fp %.2f ms value %.4e' % (d['kernels']['fp']['ms_avg'], d['value']))"
C2D_LIBRARY=$PWD/compton2d_amd/sweep/prof3/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 6 > $OUT/tr_prof.jsonl 2> $OUT/tr_prof.err \
  || { echo "tr_prof rc=$?"; tail -5 $OUT/tr_prof.err; exit 1; }
tail -1 $OUT/tr_prof.jsonl
