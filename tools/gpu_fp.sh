set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_fp.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_fp.log
exit $rc
