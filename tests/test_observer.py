"""Observer-frame SED / light-curve binning on the CPU:
the oracle restatement of the tools' per-event loop (oracle/c2d_obs_oracle.c),
the product's deck parsing, bin-edge arithmetic, file walk, normalisation and
writers (compton2d_amd/observer.py) against the reference's own pspt/plcm
output files (tests/golden/obs.npz: postprocessing/pspt.c and plcm.c run
over the reference's escape events with its mrk421 decks and two wider
decks; tests/golden/make_golden.py:make_observer).  Byte-identical text."""
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd import abi, observer

G = np.load(Path(__file__).resolve().parent / "golden" / "obs.npz", allow_pickle=False)
DECKS = sorted(k[5:] for k in G.files if k.startswith("deck_"))


def _binning(name):
    tool, deck = str(G["tool_" + name]), str(G["deck_" + name])
    return tool, (observer.parse_pspt_deck(deck) if tool == "pspt" else observer.parse_plcm_deck(deck))


def _event_dir(tmp_path):
    ev = G["events"]
    n1 = int(G["n_file1"])
    observer.write_events(tmp_path / "p001_evb.dat", ev[:n1])
    observer.write_events(tmp_path / "p002_evb.dat", ev[n1:])
    return ev


def test_event_file_round_trip(tmp_path):
    ev = _event_dir(tmp_path)
    files, factor = observer.event_files("p001_evb.dat", tmp_path)
    assert [f.name for f in files] == ["p001_evb.dat", "p002_evb.dat"]
    assert factor == 1                           # '#factor: 1' in every reference output
    back = np.concatenate([observer.read_events(f) for f in files])
    assert np.array_equal(back, ev)


def test_event_file_walk_letters(tmp_path):
    """p001..p003_evb, then p001_evc: factor counts series not restarting at 001."""
    for nm in ("p001_evb.dat", "p002_evb.dat", "p003_evb.dat", "p001_evc.dat"):
        (tmp_path / nm).write_text("")
    files, factor = observer.event_files("p001_evb.dat", tmp_path)
    assert [f.name for f in files] == ["p001_evb.dat", "p002_evb.dat", "p003_evb.dat", "p001_evc.dat"]
    assert factor == 2


@pytest.mark.parametrize("name", DECKS)
def test_oracle_and_writers_match_reference_tools(name, tmp_path):
    tool, b = _binning(name)
    ev = _event_dir(tmp_path)
    files, factor = observer.event_files(b.infile, tmp_path)
    F, F2, cnt = OL.obs_bin(b, ev, "ref")
    h = observer.Histogram(F, F2, cnt)
    out = tmp_path / "out"
    out.mkdir()
    if tool == "pspt":
        observer.write_sed(out / b.outfiles[0], b, h, factor)
    else:
        observer.write_lc(out, b, h, factor)
    want = list(G["files_" + name])
    assert sorted(p.name for p in out.iterdir()) == sorted(want)
    for f in want:
        ref = str(G["out_%s__%s" % (name, f)])
        got = (out / f).read_text()
        assert got == ref, (name, f, next((i, a, c) for i, (a, c) in enumerate(
            zip(got.splitlines(), ref.splitlines())) if a != c))
    assert cnt.sum() > (0 if "mrk421" in name else 1000)


@pytest.mark.parametrize("name", DECKS)
def test_det_oracle_bins_like_ref_oracle(name):
    """The GPU's fdlibm cos (c2d_math.h) against glibc's: same bins on these events."""
    _, b = _binning(name)
    ev = G["events"]
    a = OL.obs_bin(b, ev, "ref")
    d = OL.obs_bin(b, ev, "det")
    assert np.array_equal(a[2], d[2])
    np.testing.assert_allclose(d[0], a[0], rtol=1e-15, atol=0)


def test_binning_edges():
    b = observer.parse_pspt_deck("p001_evb.dat\n33\n1e16\nx\n30\n1.6e4\n6e4\n0.99944\n0.99964\n1\n"
                                 "1e-7\n1e10\n100\n0\nn\n")
    assert b.outfiles == ["x.dat"] and b.n_t == 30 and b.n_e == 100
    assert b.E0[0] == 1e-7 and b.E1[-1] == pytest.approx(1e10, rel=1e-12)
    assert np.array_equal(b.E0[1:], b.E1[:-1])
    lc = observer.parse_plcm_deck("")
    assert lc.mode == abi.OBS_LC and lc.n_t == 1024 and lc.n_mu == 1 and lc.n_e == 7
    assert lc.outfiles == ["lc07_ev0.dat"] and lc.dt == 7e2 and lc.t_stop == 7e4
    assert np.array_equal(lc.t1[:-1], lc.t0[1:])


def test_mrk421_sed_deck_is_the_reference_deck():
    """bench.py's C3 step bins its escapes with observer.mrk421_sed_binning():
    the deck text is the reference's postprocessing/mrk421_sed.input as the
    golden generator read it (tests/golden/obs.npz deck_sed_mrk421)."""
    assert observer.MRK421_SED_DECK == str(G["deck_sed_mrk421"])
    b = observer.mrk421_sed_binning()
    assert (b.n_t, b.n_mu, b.n_e) == (30, 1, 100) and b.outfiles == ["sed30.dat"]
