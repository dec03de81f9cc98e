# On the GPU box: pytest -m gpu, smoke(), bench, rocprof kernel-trace + PMC passes.
#   bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-cur}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== pytest gpu $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== profile $(date +%T)"
timeout -k 10 900 bash tools/gpu_profile.sh "$TAG" > gpurun_out/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof.log; exit 1; }
tail -20 gpurun_out/prof.log
