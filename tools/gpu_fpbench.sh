set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fp
timeout -k 10 300 python tools/fp_bench.py --grid 32 --reps 2 --cpu-zones 16 > gpurun_out/fp/fp_bench.json 2> gpurun_out/fp/fp_bench.err || { tail -20 gpurun_out/fp/fp_bench.err; exit 1; }
cat gpurun_out/fp/fp_bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/fp/kt" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/fp_bench.py" --grid 32 --reps 2 --cpu-zones 1 > "$GRAFT_REPO_ROOT/gpurun_out/fp/fp_bench_kt.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/fp/kt.err" || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/fp/kt.err"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/fp/kt" -name "*kernel_stats.csv" -exec head -5 {} \;
