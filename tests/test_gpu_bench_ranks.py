"""bench.py's N > 1 path on a one-GPU box: two torchrun
ranks on device 0 over gloo (C2D_ONE_GPU=1, C2D_DIST_BACKEND=gloo; RCCL
refuses two ranks on one device) against one rank with the same global
workload.  Sources are sharded by lineage, tallies all-reduced every step and
the FP update run redundantly on every rank, so the all-reduced packet-step
count of the timed steps equals the one-rank run's exactly."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out: str) -> dict:
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("workload,spinup", [("c3", 1), ("c4", 2)])
def test_two_ranks_on_one_gpu_match_one_rank(workload, spinup):
    """c3 is the default at every N; c4 (BASELINE configs[3]'s per-GPU
    load) the 32x32 C2 medium, FP off, the in-place chunked census
    (bench.py INPLACE) carried through spin-up steps."""
    common = ["--workload", workload, "--spinup", str(spinup), "--steps", "2", "--warmup", "1",
              "--no-cpu-baseline"]
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--sources", "8000000"] + common,
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-2000:]
    env = dict(os.environ, C2D_ONE_GPU="1", C2D_DIST_BACKEND="gloo")
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                          "--gpus", "2", "--sources", "4000000"] + common,
                         capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert two.returncode == 0, two.stderr[-2000:]
    a, b = _last_json(one.stdout), _last_json(two.stdout)
    assert b["n_gpus"] == 2 and a["n_gpus"] == 1
    assert b["config"]["packet_steps_timed"] == a["config"]["packet_steps_timed"] > 0
    if workload == "c4":
        assert a["config"]["census"]["layout"].startswith("chunked")
        assert b["config"]["census"]["layout"].startswith("chunked")
        assert a["config"]["census"]["records_after_spinup"] > 0
