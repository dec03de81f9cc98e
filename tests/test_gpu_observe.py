"""Observer-frame binning on the GPU (c2d_obs_*, compton2d_amd/csrc/observe.hip)
against the oracle (oracle/c2d_obs_oracle.c, pinned byte-for-byte to the
reference's pspt/plcm in tests/test_observer.py) and against the reference
tools' own output files (tests/golden/obs.npz).

Counts are exact (integer work: the bin decisions use the same fdlibm cos as
the det oracle).  The ew sums are accumulated with device atomics in an
unspecified order, so they match the tools' sequential sums to rounding:
rtol 1e-12 on the raw sums; the printed %e text (7 digits) then matches the
reference's up to a last-digit flip, checked as rtol 2e-6 per number."""
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, observer, synth
from compton2d_amd.engine import Engine, obs_engine

pytestmark = pytest.mark.gpu

G = np.load(Path(__file__).resolve().parent / "golden" / "obs.npz", allow_pickle=False)
DECKS = sorted(k[5:] for k in G.files if k.startswith("deck_"))


@pytest.fixture(scope="module")
def eng():
    e = obs_engine(0)
    yield e
    e.close()


def _binning(name):
    tool, deck = str(G["tool_" + name]), str(G["deck_" + name])
    return tool, (observer.parse_pspt_deck(deck) if tool == "pspt" else observer.parse_plcm_deck(deck))


def _check_sums(h, want):
    F, F2, cnt = want
    assert np.array_equal(h.count, cnt), np.argwhere(h.count != cnt)[:5]
    np.testing.assert_allclose(h.F, F, rtol=1e-12, atol=0)
    np.testing.assert_allclose(h.F2, F2, rtol=1e-12, atol=0)


def _same_text(got: str, ref: str):
    gl, rl = got.splitlines(), ref.splitlines()
    assert len(gl) == len(rl)
    for a, b in zip(gl, rl):
        if a == b:
            continue
        ta, tb = a.split(), b.split()
        assert len(ta) == len(tb), (a, b)
        for x, y in zip(ta, tb):
            if x != y:
                assert float(x) == pytest.approx(float(y), rel=2e-6), (a, b)


@pytest.mark.parametrize("name", DECKS)
def test_gpu_binning_matches_oracle_and_reference_files(eng, name, tmp_path):
    tool, b = _binning(name)
    ev = G["events"]
    n1 = int(G["n_file1"])
    h = observer.bin_events(eng, b, [ev[:n1], ev[n1:]])       # one launch per event file
    _check_sums(h, OL.obs_bin(b, ev, "det"))
    if tool == "pspt":
        observer.write_sed(tmp_path / b.outfiles[0], b, h, 1)
    else:
        observer.write_lc(tmp_path, b, h, 1)
    for f in G["files_" + name]:
        _same_text((tmp_path / f).read_text(), str(G["out_%s__%s" % (name, f)]))


def test_gpu_tool_drop_in(tmp_path):
    """python -m compton2d_amd.observer plcm < deck, over event files in a run dir."""
    ev = G["events"]
    n1 = int(G["n_file1"])
    observer.write_events(tmp_path / "p001_evb.dat", ev[:n1])
    observer.write_events(tmp_path / "p002_evb.dat", ev[n1:])
    for name in ("lc_wide", "sed_wide"):
        written = observer.run_tool(str(G["tool_" + name]), str(G["deck_" + name]), tmp_path)
        assert sorted(p.name for p in written) == sorted(G["files_" + name])
        for f in G["files_" + name]:
            _same_text((tmp_path / f).read_text(), str(G["out_%s__%s" % (name, f)]))


def _many_events(n, seed=3):
    """Jittered copies of the reference's events (same shape and ranges)."""
    rng = np.random.default_rng(seed)
    base = G["events"][rng.integers(0, len(G["events"]), n)].copy()
    base[:, 0] *= rng.uniform(0.5, 2.0, n)
    base[:, 1] *= 10.0 ** rng.uniform(-1, 1, n)
    base[:, 5] = np.clip(base[:, 5] + rng.normal(0, 2e-4, n), -1, 1)
    base[:, 6] = rng.uniform(0, 2 * np.pi, n)
    return base


@pytest.mark.parametrize("name", ["sed_wide", "lc_wide", "sed_overlap"])
def test_gpu_binning_large_batch(eng, name):
    """2M events: LDS-privatised (SED) and global-atomic (LC, 516 KB histogram)
    paths; sorted edges (binary search) and overlapping, unsorted energy
    regions (the tools' linear first-match scan)."""
    if name == "sed_overlap":
        b = observer.sed_binning(33., 1e16, 12, -4000., 2e4, 0.999, 1.0,
                                 ((1e-2, 1e4, 12, False), (1e-4, 1e2, 10, True), (5., 5e5, 3, False)))
        assert not np.all(np.diff(b.E0) >= 0)
    else:
        _, b = _binning(name)
    ev = _many_events(2_000_000)
    h = observer.bin_events(eng, b, [ev])
    _check_sums(h, OL.obs_bin(b, ev, "det"))
    assert h.count.sum() > 1e5


def test_gpu_bins_device_event_buffer():
    """events=None: the escape events of the last transport step, never copied
    to the host (what the text files carried)."""
    wl = synth.c2_workload(nz=3, nr=3, sources=100_000, census_capacity=400_000,
                           event_capacity=400_000)
    si = wl.step0
    si.ncycle = 1
    with Engine(wl.grid) as e:
        e.transport_step(si)
        ev = e.events()
        assert len(ev) > 10_000
        b = observer.sed_binning(33., 7.5e15, 20, -2e4, 2e4, 0.99, 1.0,
                                 ((1e-6, 1e2, 30, False), (1e2, 1e8, 30, False)))
        h = observer.bin_events(e, b, [None])
        _check_sums(h, OL.obs_bin(b, ev, "det"))
        assert h.count.sum() > 1000


@pytest.mark.parametrize("name", [n for n in DECKS if str(G["tool_" + n]) == "pspt"])
def test_gpu_pspt_deck_and_file_through_the_c_abi(eng, name, tmp_path):
    """c2d_obs_begin_pspt (pspt's dialogue parsed and turned into edges by
    the library, postprocessing/pspt.c:105-205) + c2d_obs_write_pspt (its
    file, :323-353), the drop-in shim's default event output: the reference
    pspt's own output file of the same deck and events (tests/golden/obs.npz),
    as test_gpu_binning_matches_oracle_and_reference_files checks the
    Python writer."""
    deck = str(G["deck_" + name])
    ev = G["events"]
    n1 = int(G["n_file1"])
    eng.obs_begin_pspt(deck)
    eng.obs_accumulate(ev[:n1])
    eng.obs_accumulate(ev[n1:])
    b = observer.parse_pspt_deck(deck)
    out = tmp_path / b.outfiles[0]
    eng.obs_write_pspt(str(out), factor=1)
    (f,) = G["files_" + name]
    _same_text(out.read_text(), str(G["out_%s__%s" % (name, f)]))
    with pytest.raises(Exception, match="C2D_E_ARG"):
        eng.obs_begin_pspt("p001_evb.dat\n33\n1e16\nx\n30\n1.6e4\n6e4\n0.99944\n0.99964\n1\n1e-7\n1e10\n201\n")
