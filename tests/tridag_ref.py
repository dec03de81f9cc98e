"""Pure-Python restatement of src/update2d.f:2476-2518 (`tridag`) — TEST INFRASTRUCTURE."""
import numpy as np


def tridag_ref(a, b, c, r, x_prev):
    n = len(b)
    f = np.array(x_prev, np.float64, copy=True)
    if abs(b[0]) <= 1.0e-100:          # 'Error: b(1) = 0.' -> return, f_new unchanged
        return f
    gam = np.zeros(n)
    bet = b[0]
    f[0] = r[0] / bet
    for i in range(1, n):
        gam[i] = c[i - 1] / bet
        bet = b[i] - a[i] * gam[i]
        if abs(bet) <= 1.0e-100:       # 'Error: bet = 0.' -> f_new = 0
            return np.zeros(n)
        f[i] = (r[i] - a[i] * f[i - 1]) / bet
    for i in range(n - 2, -1, -1):
        f[i] = f[i] - gam[i + 1] * f[i + 1]
        if f[i + 1] < 0.0:
            f[i + 1] = 0.0
    return f
