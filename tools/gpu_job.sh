set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -u tools/c3_bench.py --sources 20000000 --steps 90 > gpurun_out/r03a/c3_traj.jsonl 2> gpurun_out/r03a/c3_traj.err || { echo "traj failed rc=$?"; tail -5 gpurun_out/r03a/c3_traj.err; exit 1; }
tail -2 gpurun_out/r03a/c3_traj.jsonl | cut -c1-400
