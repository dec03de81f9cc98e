set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_compton.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not reference_streams" > gpurun_out/r03b/pytest.log 2>&1; rc=$?
grep -E "Compton|PASS|FAIL|Error|assert" gpurun_out/r03b/pytest.log | head -60
tail -3 gpurun_out/r03b/pytest.log
exit $rc
