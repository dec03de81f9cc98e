"""Census checkpoint files: compton2d_amd/census_io.py
against the reference's own write_cens / read_cens (src/census2d.f:1-76),
run on the same records by oracle/ref/c2d_censdrv.f (fixture
tests/golden/census_fmt.npz, made by tests/golden/make_golden.py)."""
import numpy as np
import pytest

from compton2d_amd import census_io as CI
from golden_io import GOLDEN


@pytest.fixture(scope="module")
def fmt():
    return dict(np.load(GOLDEN / "census_fmt.npz", allow_pickle=False))


def test_writer_is_byte_identical_to_reference_write_cens(fmt, tmp_path):
    d, i6 = fmt["d"], fmt["i6"]
    keys = i6[:, 5].astype(np.uint64)          # keys whose reduced form is the reference seed
    CI.write_census(tmp_path / "c.txt", d, i6[:, :5], keys)
    assert (tmp_path / "c.txt").read_bytes() == bytes(fmt["text"])


def test_reader_equals_reference_read_cens(fmt, tmp_path):
    p = tmp_path / "ref.txt"
    p.write_bytes(bytes(fmt["text"]))          # a file written by the reference
    d6, i5, keys = CI.read_census(p)
    np.testing.assert_array_equal(d6, fmt["read_d"])
    np.testing.assert_array_equal(i5, fmt["read_i"][:, :5])
    # no key file: keys derived from the 5-digit seed column and the record index
    assert keys.dtype == np.uint64 and len(set(keys.tolist())) == len(keys)
    assert CI.derive_key(fmt["read_i"][3, 5], 3) == keys[3]


def test_round_trip_keeps_keys_and_e14_7_precision(tmp_path):
    rng = np.random.default_rng(1)
    d = rng.uniform(-1, 1, (50, 6)) * 10.0 ** rng.integers(-10, 40, (50, 6))
    i5 = rng.integers(0, 99, (50, 5)).astype(np.int32)
    keys = rng.integers(0, 2 ** 63, 50).astype(np.uint64) * np.uint64(2)
    CI.write_census(tmp_path / "c.txt", d, i5, keys)
    d2, i2, k2 = CI.read_census(tmp_path / "c.txt")
    np.testing.assert_array_equal(k2, keys)
    np.testing.assert_array_equal(i2, i5)
    np.testing.assert_allclose(d2, d, rtol=5.0001e-7)     # 7 significant digits (0.ddddddd)
    assert CI.fortran_e14_7(-2.5e-101) == "-0.2500000-100"   # Ew.d drops the E for 3 digits
    assert CI.fortran_e14_7(2.5e-100) == " 0.2500000E-99"
