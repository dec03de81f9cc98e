set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Compton," $O/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
s() { python -c "import json,sys;d=json.load(open(sys.argv[1]));ps=d['config']['per_step'];print(sys.argv[1],'%.3g'%d['value'],'%.1f'%d['ms_per_step'],'g0 %.1f'%ps['transport_gen0_ms'],'all %.1f'%ps['transport_all_ms'],'cens %.3g'%ps.get('census_records',0),'frac %.3f'%d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))" $1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/e1.err || { tail -5 $O/e1.err; exit 1; }
s $O/bench_c3.json
for t in base fexp fdiv rsq1 allf; do
  lib=""; [ $t = base ] || lib=$PWD/compton2d_amd/sweep/$t/libcompton2d.so
  C2D_LIBRARY=$lib timeout -k 10 300 python bench.py --spinup 0 --steps 4 --warmup 4 --no-cpu-baseline > $O/ab_$t.json 2> $O/ab_$t.err || { tail -5 $O/ab_$t.err; exit 1; }
  s $O/ab_$t.json
done
timeout -k 10 400 python bench.py --workload c4 --steps 5 --warmup 2 > $O/bench_c4.json 2> $O/e2.err || { tail -5 $O/e2.err; exit 1; }
s $O/bench_c4.json
