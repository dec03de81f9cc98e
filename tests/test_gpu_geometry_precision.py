"""the fast build takes ONE Newton step after v_rsq_f64 /
v_rcp_f64 (transport.hip C2D_FAST_NR, fsqrt_nn / rcp_pos), 4e-15 / 2e-15
relative in isolation (test_gpu_rcp_precision.py).  The flight step's
boundary distance disbr = inout*sqrt(rbnd^2 - psq) - Eta*rpre
(src/imctrk2d.f:251-277) cancels near tangency, so the sqrt's relative error
becomes an absolute error of ~eps*rbnd in the distance.  This measures that
error on the GPU for near-tangent rays -- grazing the outer boundary from
inside (rpre -> rbnd, Eta -> 1), clipping the inner boundary (psq ->
rbnd^2, Eta < 0) -- against an 80-bit host evaluation of the same
expression from the same doubles, for the exact build's IEEE sequence and
the fast build's with one and two Newton steps (c2d_selftest_geom), and
prices it: the chance that a step's event (boundary vs census vs collision,
and so the cell it ends in) flips is the distance error over the distances
the comparison sees.  Measured on the box (r06i): the f64 formula itself is
off by up to ~7.6e6 eps*rbnd from the 80-bit value at tangency, the same in
every build; one Newton step moves the result by a few eps*rbnd from the
exact build's IEEE result.  Printed; asserted: the fast builds stay within
64 eps*rbnd of IEEE, far below the formula's own f64 error."""
import numpy as np
import pytest

from compton2d_amd.engine import device_geom

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps


def _rays(n=1 << 18, seed=5):
    rng = np.random.default_rng(seed)
    rbnd = 10.0 ** rng.uniform(14.0, 16.0, n)
    wmu = rng.uniform(-0.999, 0.999, n)
    rays = np.empty((n, 4))
    h = n // 2
    # outward, grazing the outer boundary: rpre = rbnd (1 - d), Eta -> 1
    d = 10.0 ** rng.uniform(-13.0, -1.0, h)
    rays[:h, 0] = rbnd[:h] * (1.0 - d)
    rays[:h, 1] = 1.0 - 10.0 ** rng.uniform(-14.0, -1.0, h)
    rays[:h, 3] = rbnd[:h]
    # inward, clipping the inner boundary rin = rbnd: psq = rpre^2 (1 - Eta^2) -> rin^2 from below
    rin = rbnd[h:]
    rpre = rin * (1.0 + 10.0 ** rng.uniform(-6.0, 0.0, n - h))
    sin2 = (rin / rpre) ** 2 * (1.0 - 10.0 ** rng.uniform(-14.0, -2.0, n - h))
    rays[h:, 0] = rpre
    rays[h:, 1] = -np.sqrt(1.0 - sin2)
    rays[h:, 3] = -rin
    rays[:, 2] = wmu
    return rays


def _reference(rays):
    """The same expression in 80-bit long double from the same doubles."""
    L = np.longdouble
    rpre, eta, wmu = rays[:, 0].astype(L), rays[:, 1].astype(L), rays[:, 2].astype(L)
    rbnd = np.abs(rays[:, 3]).astype(L)
    inout = np.where(rays[:, 3] < 0, L(-1), L(1))
    psq = rpre * rpre * (L(1) - eta * eta)
    dpbsq = np.maximum(rbnd * rbnd - psq, L(1.0e-6))
    disbr = inout * np.sqrt(dpbsq) - eta * rpre
    trldb = disbr / np.sqrt(L(1) - wmu * wmu)
    return disbr, trldb


def test_near_tangent_boundary_distance(capsys):
    """The formula itself, in f64 as the reference evaluates it, loses
    ~sqrt(eps)*rbnd at tangency (psq rounds before the cancellation in
    rbnd^2 - psq): every build carries that error, measured here against
    80-bit evaluation.  The Newton steps only add their own rounding on top:
    the fast builds are compared with the exact build's IEEE sequence."""
    if np.finfo(np.longdouble).eps >= EPS:
        pytest.skip("no extended long double on this host")
    rays = _rays()
    rd, rt = _reference(rays)
    scale = np.abs(rays[:, 3])
    swmu = np.sqrt(1.0 - rays[:, 2] ** 2)
    out = {nr: device_geom(nr, rays) for nr in (0, 1, 2)}
    intrinsic = np.abs(out[0][:, 0] - rd.astype(np.float64)) / scale
    res = {"f64_formula_vs_80bit": dict(max=float(intrinsic.max()) / EPS,
                                        p99=float(np.quantile(intrinsic, 0.99)) / EPS)}
    for nr, name in ((1, "fast_1N_vs_ieee"), (2, "fast_2N_vs_ieee")):
        ed = np.abs(out[nr][:, 0] - out[0][:, 0]) / scale
        et = np.abs(out[nr][:, 1] - out[0][:, 1]) * swmu / scale
        # a comparison trldb < dcen / trldb < dcol sees distances of a cell
        # (the boundary radius / 30, C3's zone size): an absolute error e
        # flips one of them with probability ~ e / that
        res[name] = dict(disbr_max=float(ed.max()) / EPS, disbr_p99=float(np.quantile(ed, 0.99)) / EPS,
                         trldb_max=float(et.max()) / EPS, flip_prob=float(30.0 * ed.mean()))
    with capsys.disabled():
        print("\nnear-tangent boundary distance, error / (eps * rbnd):",
              {k: {q: "%.3g" % v for q, v in r.items()} for k, r in res.items()})
    for name in ("fast_1N_vs_ieee", "fast_2N_vs_ieee"):
        assert res[name]["disbr_max"] < 64 and res[name]["trldb_max"] < 64, res
        assert res[name]["flip_prob"] < 1e-13, res
    # what one Newton step adds is far below what the f64 formula already carries
    assert res["fast_1N_vs_ieee"]["disbr_p99"] < 1e-3 * res["f64_formula_vs_80bit"]["p99"], res
