#!/bin/bash
# GPU-box recipes (run through gpurun from the repo root):
#   bash tools/gpu.sh <tag> <recipe> [recipe ...]
# Results go to gpurun_out/<tag>/.  Every GPU step runs under its own
# timeout; the first failing step ends the script (nothing more is started).
#
# recipes
#   tests          the whole `pytest -m gpu` suite, one process
#   tests:<files>  some test files (comma-separated, under tests/)
#   smoke          __graft_entry__.smoke()
#   bench          bench.py with the driver's defaults (C3, N=1, with cpu_baseline)
#   c3 | c3chunk | c4 | c5   bench.py workloads without cpu_baseline (STEPS/WARMUP)
#   ab:<t1>,<t2>   bench each tuning build compton2d_amd/sweep/<t>/ (tools/build_sweep.sh;
#                  "base" = the in-tree library), SPINUP/STEPS/WARMUP
#   profile        rocprofv3 kernel trace + PMC passes of the C3 bench (tools/gpu_profile.sh)
#   fp             tools/fp_bench.py off the clamp: 30x9, varied zones, memo on and off
#   fpab:<t1>,..   the fp run for each build (as ab:)
#   fpfast         the fast FP off the clamp, McDonald moment table on/off, memo warm/cold
#   fppmc          rocprofv3 kernel trace + SQ counters of that FP run (memo on)
#   fpprof         FP section timers off the clamp (sweep build "fpprof", tools/fp_prof.py)
#   trprof[:t,..]  wave section timers of the C3 run (sweep builds, default "prof"; tools/tr_prof.py)
#   n2             rehearse bench.py's N>1 path: 2 gloo ranks on device 0 vs 1 rank
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
STEPS=${STEPS:-10}; WARMUP=${WARMUP:-3}

line() {  # one-line summary of a bench JSON
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ps, c = d["config"]["per_step"], d["config"]["census"]
print(sys.argv[1], "%.4g" % d["value"], "ms %.1f" % d["ms_per_step"], "g0 %.1f" % ps["transport_gen0_ms"],
      "all %.1f" % ps["transport_all_ms"], "cens %.3g" % c["records_at_end"], "frac %.3f" % d["roofline"]["frac"],
      {k: c[k] for k in c if k.startswith("chunks") or k.startswith("last_close")},
      (d.get("cpu_baseline") or {}).get("value"))
PY
}
run() {  # run <seconds> <name> <cmd...>: stdout -> $O/<name>.out, stderr -> $O/<name>.err
  local t=$1 n=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err" || { echo "$n failed rc=$?"; tail -20 "$O/$n.err"; tail -5 "$O/$n.out"; exit 1; }
}

for r in "$@"; do
  case $r in
    tests)
      run 900 pytest python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      grep -E "passed|failed" "$O/pytest.out" | tail -3 ;;
    tests:*)
      files=$(echo "${r#tests:}" | tr ',' '\n' | sed 's#^#tests/#' | tr '\n' ' ')
      run 900 pytest_part python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread
      grep -E "passed|failed" "$O/pytest_part.out" | tail -3 ;;
    smoke)
      run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"; tail -2 "$O/smoke.out" ;;
    bench)
      run 600 bench python bench.py; line "$O/bench.out" ;;
    c3)      run 500 c3 python bench.py --steps $STEPS --warmup $WARMUP --no-cpu-baseline --no-fp-offclamp; line "$O/c3.out" ;;
    c3chunk) run 500 c3chunk python bench.py --steps $STEPS --warmup $WARMUP --no-cpu-baseline --census-inplace 1
             line "$O/c3chunk.out" ;;
    c4)      run 600 c4 python bench.py --workload c4 --steps $STEPS --warmup $WARMUP --no-cpu-baseline; line "$O/c4.out" ;;
    c5)      run 500 c5 python bench.py --workload c5 --steps $STEPS --warmup $WARMUP --no-cpu-baseline; line "$O/c5.out" ;;
    ab:*)
      for t in $(echo "${r#ab:}" | tr ',' ' '); do
        lib=""; [ "$t" = base ] || lib=$PWD/compton2d_amd/sweep/$t/libcompton2d.so
        C2D_LIBRARY=$lib run 400 "ab_$t" python bench.py --spinup "${SPINUP:-0}" --steps "${STEPS}" \
            --warmup "${WARMUP}" --no-cpu-baseline --no-fp-offclamp
        line "$O/ab_$t.out"
      done ;;
    profile)
      run 1000 profile bash tools/gpu_profile.sh "$TAG"; tail -20 "$O/profile.out" ;;
    fp)
      for m in 1 0; do
        C2D_FP_MEMO=$m run 300 "fp_memo$m" python tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 --cpu-zones 8
        tail -1 "$O/fp_memo$m.out"
      done ;;
    fpfast)  # the fast FP off the clamp: McDonald moment table on / off / with the shared memo
             # (C2D_FPF_MTAB 1 / 0 / 2), gamma_bar memo warm or emptied before every update
      for v in 1:0 1:1 0:0 0:1 2:1; do
        mt=${v%%:*}; rs=${v##*:}
        C2D_FPF_MTAB=$mt C2D_FPF_MEMO_RESET=$rs run 300 "fpfast_mt${mt}_cold${rs}" \
          python tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 --cpu-zones 8 --mode fast
        echo "fpfast mtab=$mt cold=$rs: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.2f ms (first call %.2f), f_nt dev %.1e, Te equal %s' % (d['kernel_ms'], d['kernel_ms_first_call'], d['f_nt_max_dev_vs_oracle_on_sample'], d['Te_new_equal_on_sample']))" "$O/fpfast_mt${mt}_cold${rs}.out")"
      done ;;
    fpab:*)  # tools/fp_bench.py off the clamp for each build (as ab:, memo on)
      for t in $(echo "${r#fpab:}" | tr ',' ' '); do
        lib=""; [ "$t" = base ] || lib=$PWD/compton2d_amd/sweep/$t/libcompton2d.so
        C2D_LIBRARY=$lib run 300 "fpab_$t" python tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 --cpu-zones 8
        echo "fpab_$t $(tail -1 $O/fpab_$t.out | cut -c1-200)"
      done ;;
    fppmc)   # kernel trace + SQ counters of the off-clamp FP run (memo on)
      R=$PWD; F=$R/$O/fpprof; mkdir -p "$F"
      FPB="$R/tools/fp_bench.py --nz 30 --nr 9 --vary --reps 3 --cpu-zones 1 --mode ${FPMODE:-exact}"
      ( cd /tmp && export TMPDIR=/tmp &&
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$F/kt" -o run --output-format csv -- \
            python3 $FPB > "$F/kt.out" 2> "$F/kt.err" &&
        timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
            SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d "$F/sq" -o run \
            --output-format csv -- python3 $FPB > "$F/sq.out" 2> "$F/sq.err" ) \
        || { echo "fppmc failed"; tail -5 "$F"/*.err; exit 1; }
      python3 tools/pmc_summary.py "$F" > "$F/summary.txt"; grep -E "FP kernel|fp sq|c2d_fp" "$F/summary.txt" ;;
    fpprof)  # FP section timers of the -DC2D_FP_PROF build (make FP_FLAGS=-DC2D_FP_PROF OUT=sweep/fpprof/...)
      C2D_LIBRARY=$PWD/compton2d_amd/sweep/fpprof/libcompton2d.so run 300 fpprof python tools/fp_prof.py --nz 30 --nr 9 --vary
      tail -1 "$O/fpprof.out" ;;
    trprof|trprof:*)  # section timers of -DC2D_TR_PROF builds (tools/build_sweep.sh prof:3:off:...,-DC2D_TR_PROF)
      tags=prof; [ "$r" = trprof ] || tags=$(echo "${r#trprof:}" | tr ',' ' ')
      for t in $tags; do
        C2D_LIBRARY=$PWD/compton2d_amd/sweep/$t/libcompton2d.so run 300 "trprof_$t" python tools/tr_prof.py --steps ${STEPS}
        tail -2 "$O/trprof_$t.out"
      done ;;
    n2)
      run 300 n2_w1 python -u bench.py --workload c3 --sources 40000000 --steps 3 --warmup 2 --no-cpu-baseline
      C2D_ONE_GPU=1 C2D_DIST_BACKEND=gloo run 300 n2_w2 python -u -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload c3 \
          --sources 20000000 --steps 3 --warmup 2 --no-cpu-baseline
      line "$O/n2_w1.out"; line "$O/n2_w2.out" ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
