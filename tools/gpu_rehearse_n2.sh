#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: two torchrun ranks on
# device 0 over gloo (C2D_ONE_GPU, C2D_DIST_BACKEND), against one rank with
# the same global workload.  Lineage sharding makes the packet-step counts
# agree (to the FP's summation order from step 2 on).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-n2}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --sources 40000000 --steps 3 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_w1.json 2> $OUT/w1.err || { echo "w1 rc=$?"; tail -5 $OUT/w1.err; exit 1; }
C2D_ONE_GPU=1 C2D_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
    --sources 20000000 --steps 3 --warmup 2 > $OUT/bench_w2.json 2> $OUT/w2.err \
    || { echo "w2 rc=$?"; tail -20 $OUT/w2.err; exit 1; }
python3 - <<PY
import json
a=json.load(open("$OUT/bench_w1.json")); b=json.loads(open("$OUT/bench_w2.json").read().strip().splitlines()[-1])
sa, sb = a["config"]["packet_steps_timed"], b["config"]["packet_steps_timed"]
print("world 1: %.6e packet-steps, value %.3e;  world 2 (one GPU): %.6e packet-steps, value %.3e, n_gpus %d; rel diff %.2e"
      % (sa, a["value"], sb, b["value"], b["n_gpus"], abs(sa - sb) / sa))
PY
