#!/bin/bash
# r02r: probe bundles by superposition -- GPU suite (exact kernel vs the
# oracle's bundle tracker), then the C3 A/B of occupancy/cold-path variants
# and the section timers
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02r
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest.txt 2>&1
rc=$?
tail -8 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.txt | head -20; exit $rc; }
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base n3b256 n3cc n4cc n3cr || exit 1
C2D_LIBRARY=$PWD/compton2d_amd/sweep/prof3/libcompton2d.so timeout -k 10 300 \
  python -u tools/tr_prof.py --sources 100000000 --steps 6 > $OUT/tr_prof.jsonl 2> $OUT/tr_prof.err \
  || { echo "tr_prof rc=$?"; tail -5 $OUT/tr_prof.err; exit 1; }
tail -1 $OUT/tr_prof.jsonl
