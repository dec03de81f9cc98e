"""Host timeline of the C3 bench step: wall time inside and between the
engine calls of CoupledRun.step (bench.py's build_c3, default configuration),
to locate the host time on the step's critical path (the kernel trace shows
the GPU idle between the FP update and the next step's emission tables).
usage: python tools/host_gap.py [spinup] [steps]"""
import sys
import time
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import bench
    spin = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    args = SimpleNamespace(inplace=bench.INPLACE["c3"], fp_mode="auto", host_tables=False)
    free, _ = torch.cuda.mem_get_info(dev)
    sources = bench.DEFAULT_SOURCES["c3"]
    ecap = int(2 * sources) + (1 << 20)
    side = ecap * 56 + sources * 80 + (4 << 30)
    ccap = bench.census_capacity(sources, min(bench.CENSUS_PER_SOURCE["c3"], spin + steps + 1), free, side,
                                 args.inplace)
    from compton2d_amd import abi
    eng, run, one_step, *_ = bench.build_c3(args, 0, 1, 0, dev, sources, ccap, ecap, abi.COMTOT_TABLE)
    log = []

    def wrap(obj, name):
        f = getattr(obj, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            r = f(*a, **k)
            log.append((name, t0, time.perf_counter()))
            return r
        setattr(obj, name, w)

    for n in ("volume_em", "transport_step", "tallies_raw", "fp_step", "obs_accumulate", "census_count",
              "last_event_count", "last_kernel_ms", "last_path_steps", "last_gen0_steps"):
        wrap(eng, n)
    for _ in range(spin):
        one_step()
    torch.cuda.synchronize()
    log.clear()
    t_steps = []
    for _ in range(steps):
        t0 = time.perf_counter()
        one_step()
        t_steps.append((t0, time.perf_counter()))
    base = log[0][1]
    prev = None
    for name, a, b in log:
        gap = (a - prev) * 1e3 if prev is not None else 0.0
        print("%-18s start %9.3f ms  dur %8.3f ms  gap before %7.3f ms" % (name, (a - base) * 1e3, (b - a) * 1e3, gap))
        prev = b
    for a, b in t_steps:
        print("step %.3f ms" % ((b - a) * 1e3))


if __name__ == "__main__":
    main()
