"""Print the transport kernel's resident workgroups per CU for a few LDS sizes."""
import ctypes as C
import sys
from pathlib import Path
lib = C.CDLL(str(Path(sys.argv[1] if len(sys.argv) > 1 else
                      Path(__file__).resolve().parents[1] / "compton2d_amd/libcompton2d.so")))
f = lib.c2d_transport_occupancy_fast
f.argtypes = [C.POINTER(C.c_int), C.c_size_t, C.c_int]
for kb in (16, 32, 43, 48, 57, 64, 72, 80):
    n = C.c_int()
    for trk in (0, 1):
        rc = f(C.byref(n), kb * 1024, trk)
        print("lds %d KB, tracker %d -> blocks/CU %d (rc %d)" % (kb, trk, n.value, rc))
