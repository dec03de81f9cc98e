"""BASELINE config C3 at its full size: 1e8 volume packets per step, FP on, the
fast build the bench times (compton2d_amd/synth.py c3_workload).  The oracle
cannot run this size, so the checks are properties that hold at any size:

* every census record the step wrote is counted once by the tallies the
  census write makes (transport.hip census_write, imctrk2d.f:528-578):
  npcen per cell equals the number of records in the cell, ecens per cell
  equals the sum of their weights, and n_field per (cell, E_field bin) equals
  the sum of 6.25e8 ew / xnu over the records that carry that bin — the
  device census read back record by record (c2d_census_pack) and summed
  with torch, against the fused tally buffer;
* the records are well formed: cells and bins inside the grid, weights and
  energies positive and finite.

Tolerance: npcen exact (sums of 1.0); ecens and n_field 1e-9 relative (the
same terms summed in another order, and the fast build's reciprocal-based
quotient, a few ulp per term)."""
import numpy as np
import pytest

from compton2d_amd import abi, synth
from compton2d_amd.coupled import CoupledRun
from compton2d_amd.engine import Engine

pytestmark = pytest.mark.gpu

SOURCES = 100_000_000          # BASELINE.json C3: 1e8 volume packets per step
STEPS = 3
BATCH = 50_000_000


def test_c3_full_size_census_matches_its_tallies(capsys):
    import torch
    wl = synth.c3_workload(sources=SOURCES, comtot_mode=abi.COMTOT_TABLE,
                           census_capacity=(STEPS + 1) * SOURCES,
                           event_capacity=2 * SOURCES + (1 << 20))
    eng = Engine(wl.grid)
    run = CoupledRun(eng, wl)
    for _ in range(STEPS):
        row = run.step()
    t = eng.tallies()
    nz, nr = eng.nz, eng.nr
    nc = nz * nr
    n = eng.census_count()
    assert n > SOURCES // 2
    dev = torch.device("cuda", 0)
    cnt = torch.zeros(nc, dtype=torch.float64, device=dev)
    ecens = torch.zeros(nc, dtype=torch.float64, device=dev)
    nfield = torch.zeros(nc * abi.NPHFIELD, dtype=torch.float64, device=dev)
    rec = torch.empty((min(BATCH, n), abi.CENSUS_REC_WORDS), dtype=torch.int64, device=dev)
    for first in range(0, n, BATCH):
        m = min(BATCH, n - first)
        torch.cuda.synchronize()      # the last batch's sums (torch's stream) have read `rec`
        eng.census_pack(first, m, rec.data_ptr())
        r = rec[:m]
        ew = r[:, 4].view(torch.float64)
        xnu = r[:, 5].view(torch.float64)
        jk = r[:, 6] & 0xFFFFFFFF                 # k | ie << 7 | j << 16 | efl << 23
        k = jk & 0x7F
        j = (jk >> 16) & 0x7F
        efl = (jk >> 23) & 0x1FF
        assert bool(((j >= 1) & (j <= nz) & (k >= 1) & (k <= nr)).all())
        assert bool((efl <= abi.NPHFIELD).all())
        assert bool((torch.isfinite(ew) & (ew > 0) & torch.isfinite(xnu) & (xnu > 0)).all())
        cell = (j - 1) * nr + (k - 1)
        cnt.index_add_(0, cell, torch.ones_like(ew))
        ecens.index_add_(0, cell, ew)
        has = efl > 0
        nfield.index_add_(0, cell[has] * abi.NPHFIELD + (efl[has] - 1), 6.25e8 * ew[has] / xnu[has])
    torch.cuda.synchronize()
    cnt, ecens = cnt.cpu().numpy(), ecens.cpu().numpy()
    nfield = nfield.cpu().numpy().reshape(nz, nr, abi.NPHFIELD)
    np.testing.assert_array_equal(np.asarray(t["npcen"]).reshape(nc), cnt)
    np.testing.assert_allclose(np.asarray(t["ecens"]).reshape(nc), ecens, rtol=1e-9, atol=0)
    tnf = np.asarray(t["n_field"]).reshape(nz, nr, abi.NPHFIELD)
    np.testing.assert_allclose(tnf, nfield, rtol=1e-9, atol=1e-12 * float(np.max(nfield)))
    with capsys.disabled():
        print("\nC3 full size, step %d: %d census records, %.3g packet-steps; ecens max rel %.1e, "
              "n_field max rel %.1e" % (
                  STEPS, n, row["packet_steps"],
                  float(np.max(np.abs(np.asarray(t["ecens"]).reshape(nc) - ecens) / np.maximum(ecens, 1e-300))),
                  float(np.max(np.abs(tnf - nfield) / np.maximum(nfield, 1e-300)))))
    eng.close()
