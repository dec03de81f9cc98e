#!/usr/bin/env python3
"""Observer-frame binning throughput (c2d_obs_accumulate) on one MI355X.

Workload: N escape events already resident in HBM (jittered copies of the
reference's own events, tests/golden/obs.npz), binned with the reference's
decks: `sed_wide` (pspt, 12 x 32 bins, LDS-privatised) and `lc_wide` (plcm,
1024 x 3 x 7 bins, global atomics).  Reports events/s from the HIP-event
kernel time, the HBM roofline (56 algorithmic bytes per event: 7 f64 read
once) and the C oracle (the tools' loop, 1 core) on a bounded sample.

    python tools/obs_bench.py [--events 50000000] [--reps 5] [--cpu-events 2000000]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

HBM_PEAK_GBS = 8000.0
BYTES_PER_EVENT = 56.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=50_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-events", type=int, default=2_000_000)
    args = ap.parse_args()
    import torch
    from compton2d_amd import observer
    from compton2d_amd.engine import obs_engine
    from test_gpu_observe import G, _binning, _many_events
    import oracle_lib as OL

    eng = obs_engine(0)
    n = args.events
    chunk = 5_000_000
    dev = torch.empty((n, 7), dtype=torch.float64, device="cuda:0")
    for i in range(0, n, chunk):
        m = min(chunk, n - i)
        dev[i:i + m] = torch.from_numpy(_many_events(m, seed=11 + i // chunk))
    torch.cuda.synchronize()
    out = {"events": n, "bytes_per_event": BYTES_PER_EVENT}
    for name in ("sed_wide", "lc_wide"):
        _, b = _binning(name)
        eng.obs_begin(b)
        eng.obs_accumulate_device(dev.data_ptr(), min(n, 1_000_000))      # warm-up
        eng.obs_begin(b)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.obs_accumulate_device(dev.data_ptr(), n)
        wall = time.perf_counter() - t0
        F, F2, cnt, ms = eng.obs_result()
        per = ms / args.reps
        ach = BYTES_PER_EVENT * n / (per * 1e-3) / 1e9
        out[name] = {"kernel_ms": per, "events_per_s": n / (per * 1e-3),
                     "wall_events_per_s": n * args.reps / wall,
                     "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": ach / HBM_PEAK_GBS},
                     "binned": float(cnt.sum()) / args.reps,
                     "hist_bins": b.n_t * b.n_mu * b.n_e}
        # CPU: the tools' loop (oracle, glibc cos, 1 core) on a bounded sample
        m = min(args.cpu_events, n)
        sample = dev[:m].cpu().numpy()
        t0 = time.perf_counter()
        ref = OL.obs_bin(b, sample, "ref")
        cpu = time.perf_counter() - t0
        out[name]["cpu_baseline"] = {"value": m / cpu, "unit": "events/s", "cores": 1, "kind": "port",
                                     "sample": "%d events" % m}
        # parity on the sample
        eng.obs_begin(b)
        eng.obs_accumulate_device(dev.data_ptr(), m)
        F, F2, cnt, _ = eng.obs_result()
        out[name]["sample_counts_exact"] = bool(np.array_equal(cnt, OL.obs_bin(b, sample, "det")[2]))
        out[name]["sample_F_maxrel_vs_tools"] = float(np.max(np.abs(F - ref[0]) / np.maximum(np.abs(ref[0]), 1e-300)))
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
