"""The library's host-side pspt code (compton2d_amd/csrc/pspt_host.h: the
dialogue parser and the output writer behind c2d_obs_begin_pspt /
c2d_obs_write_pspt, the shim's default event output) on the CPU, compiled
with gcc into a small harness (tests/c/pspt_wrap.c): its bin edges equal
compton2d_amd/observer.py's restatement of pspt.c:105-205 bit for bit, and
its file equals observer.write_sed byte for byte, on the reference's own
decks (tests/golden/obs.npz) and on edge cases of the dialogue (defaults,
a digit-only input series, linear and several regions, n_t above pspt's
t_max, too many channels)."""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

from compton2d_amd import observer

HERE = Path(__file__).resolve().parent
G = np.load(HERE / "golden" / "obs.npz", allow_pickle=False)


class Deck(C.Structure):
    _fields_ = [("infile", C.c_char * 64), ("outfile", C.c_char * 64),
                ("gam_bulk", C.c_double), ("rmax", C.c_double), ("t_start", C.c_double),
                ("t_end", C.c_double), ("dt", C.c_double), ("mu0", C.c_double), ("mu1", C.c_double),
                ("n_t", C.c_int), ("n_e", C.c_int),
                ("t0", C.c_double * 90), ("t1", C.c_double * 90),
                ("E0", C.c_double * 200), ("E1", C.c_double * 200)]


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = tmp_path_factory.mktemp("pspt") / "libpspt_wrap.so"
    subprocess.run(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-o", str(so), str(HERE / "c" / "pspt_wrap.c"),
                    "-lm"], check=True)
    L = C.CDLL(str(so))
    assert L.pw_sizeof() == C.sizeof(Deck)
    L.pw_parse.argtypes = [C.c_char_p, C.POINTER(Deck)]
    L.pw_write.argtypes = [C.c_char_p, C.POINTER(Deck), C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int]
    return L


DECKS = {k[5:]: str(G[k]) for k in G.files if k.startswith("deck_") and str(G["tool_" + k[5:]]) == "pspt"}
DECKS.update({
    "mrk421": observer.MRK421_SED_DECK,
    "defaults": "",
    "digits_linear": "7\n15\n1e17\nmy_sed\n12\n0\n1e5\n0.5\n1\n1\n1e-3\n1e3\n40\n1\nn\n",
    "regions": "p002_evc.dat\n10\n\n\n95\n\n\n\n\n3\n1e-6\n1e-2\n20\n0\n\n1e2\n30\n1\n\n1e9\n50\n\nn\n",
})


def _parse(lib, text):
    d = Deck()
    rc = lib.pw_parse(text.encode(), C.byref(d))
    return rc, d


@pytest.mark.parametrize("name", sorted(DECKS))
def test_pspt_dialogue_equals_observer(lib, name):
    rc, d = _parse(lib, DECKS[name])
    assert rc == 0
    b = observer.parse_pspt_deck(DECKS[name])
    assert d.infile.decode() == b.infile and d.outfile.decode() == b.outfiles[0]
    assert (d.gam_bulk, d.rmax, d.mu0, d.mu1, d.dt) == (b.gam_bulk, b.rmax, b.mu0[0], b.mu1[0], b.dt)
    assert (d.t_start, d.t_end) == (b.t_start, b.t_end)
    assert (d.n_t, d.n_e) == (b.n_t, b.n_e)
    for f, ref in (("t0", b.t0), ("t1", b.t1), ("E0", b.E0), ("E1", b.E1)):
        got = np.ctypeslib.as_array(getattr(d, f))[:len(ref)]
        assert np.array_equal(got, ref), f


@pytest.mark.parametrize("name", sorted(DECKS))
def test_pspt_file_equals_observer(lib, name, tmp_path):
    rc, d = _parse(lib, DECKS[name])
    b = observer.parse_pspt_deck(DECKS[name])
    rng = np.random.default_rng(7)
    F = rng.lognormal(30, 5, (b.n_t, b.n_e)) * (rng.random((b.n_t, b.n_e)) < 0.7)
    cnt = np.floor(rng.random((b.n_t, b.n_e)) * 1000) * (F > 0)
    lib.pw_write(str(tmp_path / "c.dat").encode(), C.byref(d), F.ctypes.data_as(C.POINTER(C.c_double)),
                 cnt.ctypes.data_as(C.POINTER(C.c_double)), 1)
    h = observer.Histogram(F[:, None, :], (F * F)[:, None, :], cnt[:, None, :])
    observer.write_sed(tmp_path / "p.dat", b, h, 1)
    assert (tmp_path / "c.dat").read_bytes() == (tmp_path / "p.dat").read_bytes()


def test_pspt_file_equals_reference_pspt_output(lib, tmp_path):
    """The reference pspt's own file for its own events (obs.npz), written by
    the library's writer from the oracle's sums of those events."""
    import oracle_lib as OL
    for name in ("sed_mrk421", "sed_wide"):
        deck = str(G["deck_" + name])
        rc, d = _parse(lib, deck)
        b = observer.parse_pspt_deck(deck)
        F, F2, cnt = OL.obs_bin(b, G["events"], "ref")
        F, cnt = np.ascontiguousarray(F[:, 0, :]), np.ascontiguousarray(cnt[:, 0, :])
        out = tmp_path / ("%s.dat" % name)
        lib.pw_write(str(out).encode(), C.byref(d), F.ctypes.data_as(C.POINTER(C.c_double)),
                     cnt.ctypes.data_as(C.POINTER(C.c_double)), 1)
        (f,) = G["files_" + name]
        assert out.read_text() == str(G["out_%s__%s" % (name, f)])


def test_pspt_too_many_channels(lib):
    rc, _ = _parse(lib, "p001_evb.dat\n33\n1e16\nx\n30\n1.6e4\n6e4\n0.99944\n0.99964\n1\n1e-7\n1e10\n201\n")
    assert rc == -1
