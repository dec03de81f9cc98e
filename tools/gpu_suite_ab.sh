#!/bin/bash
# r02x: GPU suite, then the C3 bench (tools/gpu_tr_ab.sh base)

set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r02x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $OUT/pytest.txt 2>&1
rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.txt | head -20; exit $rc; }
STEPS=4 WARMUP=4 OUT=$OUT bash tools/gpu_tr_ab.sh base || exit 1
