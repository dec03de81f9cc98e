set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_census_restart.py tests/test_gpu_sharding.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03e/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" gpurun_out/r03e/pytest.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03e/bench.json 2> gpurun_out/r03e/bench.err || { tail -5 gpurun_out/r03e/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r03e/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['config']['per_step']['transport_gen0_ms'],d['config']['per_step']['transport_all_ms'])"
timeout -k 10 400 python -u tools/census_traj.py --sources 20000000 --steps 110 > gpurun_out/r03e/c4_traj.jsonl 2> gpurun_out/r03e/c4_traj.err || { tail -5 gpurun_out/r03e/c4_traj.err; exit 1; }
tail -1 gpurun_out/r03e/c4_traj.jsonl
