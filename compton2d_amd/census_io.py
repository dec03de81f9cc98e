"""Census record files in the reference's checkpoint format.

The reference dumps each rank's census buffer with `write_cens`
(src/census2d.f:1-36) at checkpoint time (`write_record`,
src/write_record.f:429-437) and reads it back with `read_cens` (:40-76) on
restart: two formatted lines per packet,

    (6e14.7)  rpre, zpre, wmu, phi, ew, xnu          (dbufout, imctrk2d.f:558-563)
    (6i5)     jgpsp, jgplc, jgpmu, jph, kph, seed    (ibufout, imctrk2d.f:564-569)

`seed` is the packet's next RNG seed, int(fibran()*1e5) (hazard H5).  The
engine's census packets carry a 64-bit lineage key instead; it is written as
the 6th integer reduced to the reference's range (key mod 100000) and, in
full, to a companion file `<path>.keys` (little-endian uint64, one per
packet), so a restart from our own files resumes the exact histories while
files written by the reference still load (keys are then derived from the
seed column and the record index).  As in the reference, the 6 doubles keep
e14.7 precision (0.ddddddd: 7 significant digits) across a restart; the exact
lineage keys are in the `.keys` file.
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Tuple

import numpy as np

KEY_SUFFIX = ".keys"


def fortran_e14_7(x: float) -> str:
    """Fortran `E14.7` edit descriptor: [-]0.ddddddd E+xx (gfortran/flang layout)."""
    x = float(x)
    if x == 0.0:
        s = "0.0000000E+00"
        return s.rjust(14)
    if not math.isfinite(x):
        return ("NaN" if x != x else ("Infinity" if x > 0 else "-Infinity")).rjust(14)
    neg = x < 0
    m, e = "%.6e" % abs(x), 0
    mant, exp = m.split("e")
    digits = mant.replace(".", "")           # 7 significant digits d.dddddd
    e = int(exp) + 1                          # 0.ddddddd x 10^e
    body = "0." + digits
    if abs(e) <= 99:
        es = "E%+03d" % e
    else:
        es = "%+04d" % e                       # Ew.d with a 3-digit exponent drops the E
    s = ("-" if neg else "") + body + es
    return s.rjust(14)


def fortran_i5(v: int) -> str:
    s = "%d" % int(v)
    return s.rjust(5) if len(s) <= 5 else "*****"


def derive_key(seed: int, index: int) -> int:
    """Lineage key for a census record that has only the reference's 5-digit
    seed (files written by the reference): splitmix64 of (seed, index)."""
    z = (int(seed) * 0x9E3779B97F4A7C15 + int(index) + 0x5EEDC2D) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def write_census(path, d6: np.ndarray, i5: np.ndarray, keys: np.ndarray) -> None:
    """write_cens (src/census2d.f:21-28) for an engine census export."""
    d6 = np.asarray(d6, np.float64).reshape(-1, 6)
    i5 = np.asarray(i5, np.int64).reshape(-1, 5)
    keys = np.asarray(keys, np.uint64).reshape(-1)
    n = len(keys)
    assert d6.shape[0] == n and i5.shape[0] == n
    lines = []
    for r in range(n):
        lines.append("".join(fortran_e14_7(v) for v in d6[r]))
        ints = list(i5[r]) + [int(keys[r] % np.uint64(100000))]
        lines.append("".join(fortran_i5(v) for v in ints))
    Path(path).write_text("".join(s + "\n" for s in lines))
    keys.astype("<u8").tofile(str(path) + KEY_SUFFIX)


def read_census(path) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """read_cens (src/census2d.f:61-68): returns d6 [n,6], i5 [n,5], keys [n]."""
    lines = Path(path).read_text().splitlines()
    lines = [s for s in lines if s.strip()]
    n = len(lines) // 2
    d6 = np.empty((n, 6))
    i6 = np.empty((n, 6), np.int64)
    for r in range(n):
        a, b = lines[2 * r], lines[2 * r + 1]
        for c in range(6):
            f = a[14 * c:14 * (c + 1)].strip()
            if "E" not in f.upper() and ("+" in f[1:] or "-" in f[1:]):   # 3-digit exponent
                k = max(f.rfind("+"), f.rfind("-"))
                f = f[:k] + "E" + f[k:]
            d6[r, c] = float(f.replace("D", "E"))
            i6[r, c] = int(b[5 * c:5 * (c + 1)])
    kp = Path(str(path) + KEY_SUFFIX)
    if kp.exists():
        keys = np.fromfile(str(kp), "<u8")
        assert keys.size == n, "census key file does not match the record file"
    else:
        keys = np.array([derive_key(i6[r, 5], r) for r in range(n)], np.uint64)
    return d6, i6[:, :5].astype(np.int32), keys
