import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / 'tests')]
import numpy as np
from compton2d_amd.engine import device_mcdonald
z = np.array([0.5, 1.0, 2.0, 5.0, 10.0, 20.0, 50.0])
K2, K3, cyc = device_mcdonald(z)
K2, K3, cyc2 = device_mcdonald(z)
print(list(zip(z.tolist(), cyc.tolist(), cyc2.tolist())))
