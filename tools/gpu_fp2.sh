set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_fp.log 2>&1 || { tail -30 gpurun_out/pytest_fp.log; exit 1; }
tail -2 gpurun_out/pytest_fp.log
timeout -k 10 300 python tools/fp_bench.py --grid 32 --reps 2 --cpu-zones 16 > gpurun_out/fp/fp_bench.json 2> gpurun_out/fp/fp_bench.err || { tail -20 gpurun_out/fp/fp_bench.err; exit 1; }
cat gpurun_out/fp/fp_bench.json
