"""Emission/absorption tables on the GPU (c2d_volume_em, csrc/vem.hip)
against the oracle (oracle/c2d_vem_oracle.c, det math: bit-identical) and
against the reference's own tables (the golden runs' imcgen2d output, and
volume_em through oracle/ref/c2d_vemdrv.f in tests/test_vem_oracle.py)."""
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, synth
from compton2d_amd.engine import Engine
from golden_io import GoldenCase
from test_vem_oracle import golden_state

pytestmark = pytest.mark.gpu

V = np.load(Path(__file__).resolve().parent / "golden" / "vem.npz", allow_pickle=False)
KEYS = ("kappa_tot", "eps_tot", "eps_th", "B_field", "Eloss_sy", "Eloss_cy", "Eloss_th", "Eloss_tot",
        "E_ph")


def _same(g, o):
    for k in KEYS:
        assert np.array_equal(g[k], o[k]), (k, np.argwhere(g[k] != o[k])[:4])


@pytest.mark.parametrize("case", ["ssc_tau", "grid3x4", "ec_lower"])
def test_gpu_vem_golden_runs(case):
    gc = GoldenCase(case)
    st = golden_state(gc)
    dt = gc.meta["step0"]["dt"]
    with Engine(gc.grid()) as e:
        g = e.volume_em(dt, st)
    _same(g, OL.vem_step(gc.grid(), dt, st, flavor="det"))
    # and the reference imcgen2d's own tables
    np.testing.assert_allclose(g["kappa_tot"], gc.a["in0_kappa_tot"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(g["eps_tot"], gc.a["in0_eps_tot"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(g["eps_th"], gc.a["in0_eps_th"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(g["Eloss_tot"], gc.a["in0_Eloss_tot"], rtol=1e-13, atol=0)
    np.testing.assert_allclose(g["Eloss_th"], gc.a["in0_Eloss_th"], rtol=1e-6, atol=0)


def _random_state(nz, nr, seed=5):
    """Every branch: Theta below/above 0.2, ep_switch 0/1/2, absorbed and thin
    energies, nu <= nu_p; electron spectra of the reference's fixtures."""
    rng = np.random.default_rng(seed)
    f = V["f_nt"][rng.integers(0, len(V["f_nt"]), nz * nr)].reshape(nz, nr, -1)
    return dict(tea=10 ** rng.uniform(0.5, 3.0, (nz, nr)), tna=10 ** rng.uniform(0.5, 3.0, (nz, nr)),
                n_e=10 ** rng.uniform(0.0, 11.0, (nz, nr)), B_field=10 ** rng.uniform(-2, 2.5, (nz, nr)),
                f_pair=rng.uniform(0, 0.1, (nz, nr)), zsurf=10 ** rng.uniform(30, 33, (nz, nr)),
                vol=10 ** rng.uniform(44, 47, (nz, nr)), f_nt=f,
                ep_switch=rng.integers(0, 3, (nz, nr)).astype(np.int32))


def test_gpu_vem_random_cells_bit_exact():
    wl = synth.c2_workload(nz=6, nr=5, sources=1)
    g = wl.grid
    g.gnt = V["gnt"]
    st = _random_state(6, 5)
    with Engine(g) as e:
        r = e.volume_em(7.8e3, st)
        ms = e.last_vem_ms()
    _same(r, OL.vem_step(g, 7.8e3, st, flavor="det"))
    assert (st["ep_switch"] != 0).any() and ms > 0


def test_gpu_vem_c2_grid_matches_oracle_sample():
    """The benchmark's 32x32 medium: every cell on the GPU, oracle on a sample."""
    wl = synth.c2_workload(nz=32, nr=32, sources=1)
    g = wl.grid
    st = _random_state(32, 32, seed=9)
    with Engine(g) as e:
        r = e.volume_em(wl.dt, st)
    sub = {k: (v[:2] if isinstance(v, np.ndarray) else v) for k, v in st.items()}
    g2 = synth.c2_workload(nz=32, nr=32, sources=1).grid
    g2.nz = 2
    g2.z = g.z[:2]
    o = OL.vem_step(g2, wl.dt, sub, flavor="det")
    for k in KEYS[:-1]:
        assert np.array_equal(r[k][:2], o[k]), k
