"""McDonald's K2/K3 series on the GPU (c2d_wave.hpp mcdonald23_w, used by the
FP and emission-table kernels) against the oracle's sequential McDonald
(oracle/c2d_fp_oracle.c, det math; src/volume2d.f:598-626): bit-identical over
the arguments the temperature searches visit (z = 1/Theta)."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as OL
from compton2d_amd.engine import device_mcdonald

pytestmark = pytest.mark.gpu


def test_gpu_mcdonald_bit_exact():
    z = np.concatenate([np.geomspace(0.05, 60.0, 97), [1.0 / 0.2, 1.0 / 2.0, 1.0 / 0.20000000298]])
    K2, K3, cyc = device_mcdonald(z)
    lib = OL.load("det")
    lib.c2o_mcdonald.restype = C.c_double
    lib.c2o_mcdonald.argtypes = [C.c_double, C.c_double]
    for i, zz in enumerate(z):
        assert K2[i] == lib.c2o_mcdonald(2.0, zz), zz
        assert K3[i] == lib.c2o_mcdonald(3.0, zz), zz
    print("shader cycles per K2/K3 pair: min %.0f median %.0f max %.0f" %
          (cyc.min(), np.median(cyc), cyc.max()))
