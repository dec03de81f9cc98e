"""BASELINE config C3 (the Mrk 421 SSC deck, FP on) on the GPU, against the
oracle and the reference run on that deck (tests/golden/c3_mrk421.npz).

* exact transport kernel vs the oracle (lineage RNG, det math) on the
  reference's C3 step inputs: tests/test_gpu_parity.py (c3_mrk421 is one of
  golden_io.CASES), bit-identical histories;
* c2d_fp_step on the reference's C3 FP inputs (all 270 zones): bit-identical
  to the det-math oracle on sampled zones, Te_new equal to the reference's,
  f_nt within 1e-10;
* c2d_volume_em on the FP-updated C3 state (the step-2 tables): equal to the
  det oracle bit for bit, within 1e-12 of the reference's kappa/eps_tot;
* the coupled step chained on the device (transport -> tallies -> FP
  reading n_field/ecens from the device buffer) equals the same chain run by
  the oracle (lineage transport + FP);
* the device-resident coupled loop (compton2d_amd/coupled.py: tables and
  electrons never leave the GPU) equals the host-array loop.
"""
import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, synth
from compton2d_amd.coupled import CoupledRun
from compton2d_amd.engine import Engine
from golden_io import CoupledGoldenCase
from test_c3 import SAMPLE, ZONE_KEYS

pytestmark = pytest.mark.gpu


def case():
    return CoupledGoldenCase("c3_mrk421")


def test_gpu_c3_fp_bitwise_vs_oracle_and_reference():
    gc = case()
    eng = Engine(gc.grid(device=0))
    eng.fp_set_config(gc.constants())
    for n in gc.fp_steps:
        fi = gc.fp_in(n)
        g = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
        o = OL.fp_step(gc.grid(), gc.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                       flavor="det", cells=SAMPLE)
        for cell in SAMPLE:
            j, k = divmod(cell, gc.nr)
            for key in ZONE_KEYS + ("zone_diag",):
                np.testing.assert_array_equal(g[key][j, k], o[key][j, k],
                                              err_msg="step %d zone (%d,%d) %s" % (n, j, k, key))
        ref = gc.fp_out(n)
        np.testing.assert_array_equal(g["Te_new"], ref["Te_new"])
        np.testing.assert_array_equal(g["tea"], ref["tea"])
        assert np.max(np.abs(g["f_nt"] - ref["f_nt"])) <= 1e-10 * np.max(np.abs(ref["f_nt"]))
        for key in ("E_tot_old", "E_tot_new", "hr_total"):
            assert abs(g[key] - ref[key]) <= 1e-9 * abs(ref[key]), (n, key)
    assert eng.last_fp_ms() > 0
    eng.close()


def test_gpu_c3_tables_from_fp_state():
    gc = case()
    wl = synth.c3_workload(sources=gc.meta["case"]["nst"] // 2)
    fo = gc.fp_out(1)
    st = dict(wl.fixed, tea=fo["tea"], n_e=fo["n_e"], f_nt=fo["f_nt"])
    dt = gc.meta["step2"]["dt"]
    with Engine(gc.grid(device=0)) as e:
        g = e.volume_em(dt, st)
    o = OL.vem_step(gc.grid(), dt, st, flavor="det")
    for k in ("kappa_tot", "eps_tot", "eps_th", "Eloss_tot", "Eloss_sy", "B_field"):
        assert np.array_equal(g[k], o[k]), k
    np.testing.assert_allclose(g["kappa_tot"], gc.a["in2_kappa_tot"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(g["eps_tot"], gc.a["in2_eps_tot"], rtol=1e-12, atol=0)


def test_gpu_c3_transport_then_fp_from_device_tallies():
    """Step 1 of the C3 run: exact transport on the reference's inputs, then
    FP_calc reading the device tallies; the oracle runs the same chain."""
    gc = case()
    grid = gc.grid(comtot_mode=abi.COMTOT_EXACT, device=0)
    eng = Engine(grid)
    eng.fp_set_config(gc.constants())
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in (0, 1):
        si = gc.step_inputs(n)
        eng.transport_step(si)
        assert orc.step(si) == 0
    to = orc.split()
    fi = gc.fp_in(1)
    dev = dict(fi, n_field=None, ecens=None)
    g = eng.fp_step(1, fi["time"], fi["dt"], dev, fi)
    host = dict(fi, n_field=np.asarray(to["n_field"]).reshape(gc.nz, gc.nr, abi.NPHFIELD),
                ecens=np.asarray(to["ecens"]).reshape(gc.nz, gc.nr))
    o = OL.fp_step(gc.grid(), gc.constants(), 1, fi["time"], fi["dt"], host, fi, flavor="det",
                   cells=SAMPLE)
    for cell in SAMPLE:
        j, k = divmod(cell, gc.nr)
        # the device n_field sums by atomics (order differs from the oracle at
        # 1e-16); FP_calc carries that through thousands of sub-steps
        np.testing.assert_allclose(g["f_nt"][j, k], o["f_nt"][j, k], rtol=1e-8,
                                   atol=1e-12 * np.max(o["f_nt"][j, k]))
        assert abs(g["Te_new"][j, k] - o["Te_new"][j, k]) <= 1e-8 * o["Te_new"][j, k]
    eng.close()
    orc.close()


def test_gpu_c3_device_resident_loop_equals_host_loop():
    """compton2d_amd/coupled.py with tables/electrons on the device vs the
    same loop through host arrays: same kernels, same inputs, so the same
    electron state up to the atomic summation order of the tallies."""
    runs = []
    for dev in (True, False):
        wl = synth.c3_workload(sources=200_000, comtot_mode=abi.COMTOT_TABLE)
        eng = Engine(wl.grid)
        run = CoupledRun(eng, wl, device_resident=dev)
        rows = [run.step() for _ in range(3)]
        f, p = run.electrons()
        runs.append((rows, f, p, dict(run.state)))
        eng.close()
    (ra, fa, pa, sa), (rb, fb, pb, sb) = runs
    for a, b in zip(ra, rb):
        assert a["volume_packets"] == b["volume_packets"]
        assert abs(a["packet_steps"] - b["packet_steps"]) <= 1e-3 * b["packet_steps"]
    np.testing.assert_allclose(fa, fb, rtol=1e-6, atol=1e-12 * np.max(np.abs(fb)))
    np.testing.assert_allclose(pa, pb, rtol=1e-6, atol=1e-12)
    np.testing.assert_array_equal(sa["tea"], sb["tea"])
    assert rb[-1]["aborted"] == 0 and ra[-1]["aborted"] == 0
    assert ra[-1]["mean_Te"] > 1.0e3          # FP_calc heats past the clamp, as the reference


@pytest.mark.parametrize("mode", [abi.COMTOT_EXACT, abi.COMTOT_TABLE])
def test_gpu_c3_sed_binned_on_device_equals_oracle_binning(mode):
    """C3's named output (postprocessing/mrk421_sed.input through pspt.c:245-294):
    the step's escapes binned on the device straight from the event buffer
    (c2d_obs_accumulate(ctx, NULL, 0), as bench.py's C3 step does) equal the
    oracle's binning of the same events downloaded (counts exact, ew sums to
    atomic order), for the deck's own binning and for a wide window that every
    event of the golden's first steps falls into (the deck's window opens at
    t_obs = 1.6e4 s, later than these steps' escapes reach)."""
    from compton2d_amd import observer
    gc = case()
    eng = Engine(gc.grid(comtot_mode=mode, device=0))
    wide = observer.sed_binning(n_t=4, t_start=0.0, t_end=4.0e5, mu_min=-1.0, mu_max=1.0)
    eng.transport_step(gc.step_inputs(0))        # step 0 only fills the census
    for n in (1, 2):
        eng.transport_step(gc.step_inputs(n))
        ev = eng.events()
        assert len(ev) > 100
        for b in (observer.mrk421_sed_binning(), wide):
            eng.obs_begin(b)
            eng.obs_accumulate(None)
            F, F2, cnt, ms = eng.obs_result()
            oF, oF2, ocnt = OL.obs_bin(b, ev, "det")
            np.testing.assert_array_equal(cnt, ocnt)
            np.testing.assert_allclose(F, oF, rtol=1e-12, atol=0)
            np.testing.assert_allclose(F2, oF2, rtol=1e-12, atol=0)
            assert ms > 0
        assert cnt.sum() > 0.5 * len(ev)       # the wide window holds the step's escapes
    eng.close()


def test_gpu_c3_fp_fast_within_tolerance():
    """C2D_FP_FAST on the reference's C3 FP inputs (all 270 zones on the GPU,
    sampled zones against the det oracle): the tolerance of
    tests/test_gpu_fp.py, and Te_new equal to the reference's."""
    from test_gpu_fp import fast_vs_oracle
    gc = case()
    eng = Engine(gc.grid(device=0))
    eng.fp_set_config(gc.constants())
    eng.fp_set_mode(abi.FP_FAST)
    for n in gc.fp_steps:
        fi = gc.fp_in(n)
        g = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
        o = OL.fp_step(gc.grid(), gc.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                       flavor="det", cells=SAMPLE)
        js, ks = np.divmod(np.array(SAMPLE), gc.nr)
        gs = {k: (np.asarray(v)[js, ks] if np.ndim(v) >= 2 else v) for k, v in g.items()}
        os_ = {k: (np.asarray(v)[js, ks] if np.ndim(v) >= 2 else v) for k, v in o.items()}
        for k in ("E_tot_old", "E_tot_new", "hr_total"):      # whole-grid sums: only sampled zones in o
            gs.pop(k), os_.pop(k)
        for k in ("Te_new", "tea", "gmin", "gmax", "p_nth"):
            np.testing.assert_array_equal(gs[k], os_[k], err_msg=k)
        for k in ("f_nt", "Pnt"):
            d = np.max(np.abs(gs[k] - os_[k])) / np.max(np.abs(os_[k]))
            assert d <= 1e-10, (n, k, d)
        np.testing.assert_array_equal(g["Te_new"], gc.fp_out(n)["Te_new"])
    eng.close()


def _expected_auto(tea_in, last_max_steps):
    """C2D_FP_AUTO's rule (include/compton2d.h): exact iff every zone's tea sits
    on the clamp (<= 5 or >= 1000 keV) and the last update's slowest zone took
    <= C2D_FP_AUTO_STEPS (64) sub-steps."""
    on = np.all((tea_in <= 5.0) | (tea_in >= 1000.0))
    return abi.FP_EXACT if on and (last_max_steps is None or last_max_steps <= 64) else abi.FP_FAST


def test_gpu_c3_fp_auto_mode_switches_and_stays_in_tolerance(capsys):
    """C2D_FP_AUTO on the C3 deck's FP inputs, then on the same grid with the
    zones taken off the clamp (tea varied per zone, the fp_bench --vary
    recipe): the mode follows the rule, each result equals the det oracle
    bit for bit (exact) or within tests/test_gpu_fp.py's tolerance (fast)."""
    from test_gpu_fp import fast_vs_oracle
    gc = case()
    eng = Engine(gc.grid(device=0))
    eng.fp_set_config(gc.constants())
    eng.fp_set_mode(abi.FP_AUTO)
    assert eng.last_fp_mode() == -1
    js, ks = np.divmod(np.array(SAMPLE), gc.nr)
    cell = np.arange(gc.nz * gc.nr, dtype=np.float64).reshape(gc.nz, gc.nr)
    off = dict(gc.fp_in(2), tea=300.0 * (1.0 + 0.007 * (cell % 41)))   # every zone off the clamp
    calls = [("step1", gc.fp_in(1)), ("step2", gc.fp_in(2)), ("step2 again", gc.fp_in(2)),
             ("off clamp", off), ("step2 back", gc.fp_in(2)), ("step2 settled", gc.fp_in(2))]
    last_steps, log = None, []
    for label, fi in calls:
        want = _expected_auto(np.asarray(fi["tea"]), last_steps)
        g = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
        got = eng.last_fp_mode()
        log.append((label, abi.FP_MODE_NAMES[got], float(np.max(g["zone_diag"][..., 5])), eng.last_fp_ms()))
        assert got == want, (label, got, want)
        o = OL.fp_step(gc.grid(), gc.constants(), fi["ncycle"], fi["time"], fi["dt"], fi, fi,
                       flavor="det", cells=SAMPLE)
        gs = {k: (np.asarray(v)[js, ks] if np.ndim(v) >= 2 else v) for k, v in g.items()}
        os_ = {k: (np.asarray(v)[js, ks] if np.ndim(v) >= 2 else v) for k, v in o.items()}
        for k in ("E_tot_old", "E_tot_new", "hr_total"):
            gs.pop(k), os_.pop(k)
        if got == abi.FP_EXACT:
            for k in ZONE_KEYS:
                np.testing.assert_array_equal(gs[k], os_[k], err_msg="%s %s" % (label, k))
        else:
            for k in ("Te_new", "tea", "gmin", "gmax", "p_nth"):
                np.testing.assert_array_equal(gs[k], os_[k], err_msg="%s %s" % (label, k))
            for k in ("f_nt", "Pnt"):
                assert np.max(np.abs(gs[k] - os_[k])) <= 1e-10 * np.max(np.abs(os_[k])), (label, k)
        last_steps = float(np.max(g["zone_diag"][..., 5]))
    with capsys.disabled():
        print("\nC2D_FP_AUTO on C3: " + "; ".join("%s: %s (max %d sub-steps, %.2f ms)" % x for x in log))
    modes = [m for _, m, _, _ in log]
    assert "exact" in modes and "fast" in modes
    assert modes[3] == "fast" and modes[-1] == "exact"
    eng.close()


def test_gpu_coupled_run_logs_fp_mode():
    """CoupledRun's default C2D_FP_AUTO on the C3 workload: every step with an
    FP update logs the mode it ran; the coupled run reaches the clamp and then
    runs the exact kernel (C3's steady state, the bench's timed steps)."""
    wl = synth.c3_workload(sources=100_000, comtot_mode=abi.COMTOT_TABLE)
    eng = Engine(wl.grid)
    run = CoupledRun(eng, wl)
    rows = [run.step() for _ in range(5)]
    assert rows[0]["fp_mode"] is None                        # ncycle = 0: no update
    assert all(r["fp_mode"] in ("exact", "fast") for r in rows[1:])
    assert rows[-1]["fp_mode"] == "exact" and rows[-1]["mean_Te"] > 1.0e3
    eng.close()
