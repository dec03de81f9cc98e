"""compton2d_amd — MI355X-native Implicit Monte Carlo Compton transport engine.

Hot path of bbw7561135/Compton2d (photon-packet tracking imctrk2d and its
census/volume/surface drivers, tally reductions, Fokker-Planck tridiagonal
solve) as hand-written HIP kernels for gfx950 behind the C-ABI in
include/compton2d.h.  See DESIGN.md.
"""
__version__ = "0.1.0"
