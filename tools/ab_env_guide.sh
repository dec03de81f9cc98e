set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for v in 1 0 1 0; do
  C2D_CDF_GUIDE_OFF=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp-offclamp > $O/guide_off$v.out 2> $O/guide_off$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ps=d['config']['per_step']; print(sys.argv[1], '%.4g'%d['value'], 'ms %.2f'%d['ms_per_step'], 'g0 %.2f'%ps['transport_gen0_ms'], 'tr %.2f'%(1e3*ps['transport_s']))" $O/guide_off$v.out
done
