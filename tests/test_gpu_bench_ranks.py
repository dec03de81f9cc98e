"""bench.py's N > 1 path on a one-GPU box: two torchrun
ranks on device 0 over gloo (C2D_ONE_GPU=1, C2D_DIST_BACKEND=gloo; RCCL
refuses two ranks on one device) against one rank with the same global
workload.  Sources are sharded by lineage, tallies all-reduced every step and
the FP update run redundantly on every rank, so the all-reduced packet-step
count of the timed steps equals the one-rank run's exactly, and the results
(bench.py --dump) agree to the order of the floating-point sums: the last
timed step's all-reduced tally buffer (edep, ecens, n_field, fout, edout, ...)
and, on C3, the timed steps' on-device SED summed over ranks to 1e-11, the
FP-updated electron state (f_nt, Pnt) to the fast FP tolerance (1e-10 of the
spectrum's maximum) with tea and Te_new equal, both ranks holding the same
state (src/update2d.f:1958-1973: what the per-step all-reduce keeps equal)."""
import numpy as np
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
def test_two_ranks_on_one_gpu_match_one_rank(workload, spinup, tmp_path):
    """c3 is the default at every N; c4 (BASELINE configs[3]'s per-GPU
    load) the 32x32 C2 medium, FP off, the in-place chunked census
    (bench.py INPLACE) carried through spin-up steps."""
    common = ["--workload", workload, "--spinup", str(spinup), "--steps", "2", "--warmup", "1",
              "--no-cpu-baseline", "--no-fp-offclamp"]
    d1, d2 = tmp_path / "one", tmp_path / "two"
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--sources", "8000000",
                          "--dump", str(d1)] + common,
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-2000:]
    env = dict(os.environ, C2D_ONE_GPU="1", C2D_DIST_BACKEND="gloo")
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                          "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                          "--gpus", "2", "--sources", "4000000", "--dump", str(d2)] + common,
                         capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert two.returncode == 0, two.stderr[-2000:]
    a, b = _last_json(one.stdout), _last_json(two.stdout)
    assert b["n_gpus"] == 2 and a["n_gpus"] == 1
    assert b["config"]["packet_steps_timed"] == a["config"]["packet_steps_timed"] > 0
    if workload == "c4":
        assert a["config"]["census"]["layout"].startswith("chunked")
        assert b["config"]["census"]["layout"].startswith("chunked")
        assert a["config"]["census"]["records_after_spinup"] > 0
    _compare_results(workload, d1, d2)


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def _compare_results(workload, d1, d2):
    from compton2d_amd import abi
    a = np.load(d1 / "rank0.npz")
    b0, b1 = np.load(d2 / "rank0.npz"), np.load(d2 / "rank1.npz")
    nz, nr = (30, 9) if workload == "c3" else (32, 32)
    ta = abi.split_tallies(a["tallies"], nz, nr, 1)
    tb = abi.split_tallies(b0["tallies"], nz, nr, 1)
    # both ranks hold the all-reduced buffer
    np.testing.assert_array_equal(b0["tallies"], b1["tallies"])
    for k in ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in"):
        ref = np.asarray(ta[k], float)
        assert np.allclose(tb[k], ref, rtol=1e-11, atol=1e-13 * max(np.abs(ref).max(), 1e-300)), \
            (workload, k, _rel(tb[k], ref))
    np.testing.assert_array_equal(tb["counters"][:abi.CNT_GENS], ta["counters"][:abi.CNT_GENS])
    if workload != "c3":
        return
    # the timed steps' SED: each rank bins its own escapes
    np.testing.assert_array_equal(b0["sed_count"] + b1["sed_count"], a["sed_count"])
    for k in ("sed_F", "sed_F2"):
        ref = a[k]
        assert np.allclose(b0[k] + b1[k], ref, rtol=1e-11, atol=1e-13 * ref.max()), (k, _rel(b0[k] + b1[k], ref))
    assert a["sed_count"].sum() > 0
    # the redundant FP update: every rank the same state, equal to one rank's
    for k in ("f_nt", "Pnt", "tea", "Te_new"):
        np.testing.assert_array_equal(b0[k], b1[k], err_msg=k)
    np.testing.assert_array_equal(b0["tea"], a["tea"])
    np.testing.assert_array_equal(b0["Te_new"], a["Te_new"])
    for k in ("f_nt", "Pnt"):
        assert _rel(b0[k], a[k]) <= 1e-10, (k, _rel(b0[k], a[k]))
