set -o pipefail
mkdir -p gpurun_out/r07z
for m in exact fast exact fast; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp-offclamp --fp-mode $m > gpurun_out/r07z/c3_$m.json 2> gpurun_out/r07z/c3_$m.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ps=d['config']['per_step']
print(sys.argv[2], '%.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'fp_s %.3f ms' % (1e3*ps['fp_s']), 'fp_kernel %.3f' % ps['fp_kernel_ms'], 'Te %.2f' % ps['mean_Te'])" gpurun_out/r07z/c3_$m.json $m
done
