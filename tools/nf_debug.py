"""Census records vs the n_field tally after coupled C3 steps (diagnostics for
tests/test_gpu_fullsize.py):  python tools/nf_debug.py [sources] [steps]"""
import sys
from pathlib import Path
sys.path[:0] = [str(Path(__file__).resolve().parents[1])]
import numpy as np
import torch
from compton2d_amd import abi, synth
from compton2d_amd.coupled import CoupledRun
from compton2d_amd.engine import Engine

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1
wl = synth.c3_workload(sources=S, comtot_mode=abi.COMTOT_TABLE, census_capacity=(N + 1) * S,
                       event_capacity=2 * S + (1 << 20))
eng = Engine(wl.grid)
run = CoupledRun(eng, wl)
for _ in range(N):
    run.step()
t = eng.tallies()
nz, nr = eng.nz, eng.nr
nc = nz * nr
n = eng.census_count()
rec = torch.empty((n, 8), dtype=torch.int64, device="cuda")
eng.census_pack(0, n, rec.data_ptr())
ew = rec[:, 4].view(torch.float64); xnu = rec[:, 5].view(torch.float64)
jk = rec[:, 6] & 0xFFFFFFFF
k = jk & 0x7F; j = (jk >> 16) & 0x7F; efl = (jk >> 23) & 0x1FF; ie = (jk >> 7) & 0x1FF
cell = (j - 1) * nr + (k - 1)
nf = torch.zeros(nc * 400, dtype=torch.float64, device="cuda")
has = efl > 0
nf.index_add_(0, cell[has] * 400 + (efl[has] - 1), 6.25e8 * ew[has] / xnu[has])
nf = nf.cpu().numpy().reshape(nz, nr, 400)
tn = np.asarray(t["n_field"]).reshape(nz, nr, 400)
print("records", n, "with efl", int(has.sum()), "npcen sum", float(np.sum(t["npcen"])))
print("total tally %.6e  records %.6e" % (tn.sum(), nf.sum()))
Ef = np.asarray(wl.grid.E_field)
egg = Ef[0] ** 2 / Ef[1]
x = xnu.cpu().numpy(); e = efl.cpu().numpy()
print("xnu > egg_min:", int((x > egg).sum()), " efl>0:", int((e > 0).sum()))
# the record's efl against a lookup of its xnu on E_field (first i with x < E[i+1], 1-based)
idx = np.searchsorted(Ef, x, side="right")          # number of edges <= x
look = np.clip(idx, 1, 400)
sel = e > 0
print("efl == lookup:", int((e[sel] == look[sel]).sum()), "of", int(sel.sum()),
      " efl-lookup histogram:", np.unique((e[sel] - look[sel]).clip(-5, 5), return_counts=True))
per_bin_t = tn.sum(axis=(0, 1)); per_bin_r = nf.sum(axis=(0, 1))
bad = np.where(~np.isclose(per_bin_t, per_bin_r, rtol=1e-9, atol=0))[0]
print("bins differing:", len(bad), bad[:20])
for b in bad[:8]:
    print(" bin %d tally %.4e records %.4e" % (b, per_bin_t[b], per_bin_r[b]))
per_cell_t = tn.sum(axis=2).ravel(); per_cell_r = nf.sum(axis=2).ravel()
print("cells differing:", int((~np.isclose(per_cell_t, per_cell_r, rtol=1e-9)).sum()), "of", nc)
eng.close()
