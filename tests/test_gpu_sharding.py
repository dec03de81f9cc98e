"""Multi-GPU decomposition of the HIP path, run on one GPU.

* Lineage sharding: contexts with (rank, world) =
  (0,2), (1,2), (0,3), (1,3), (2,3) track the sources g with g % world ==
  rank and their own census; per step, their tallies summed over the ranks
  equal the world-1 run's (counters bit for bit, f64 tallies to the atomic
  summation order), and the union of their census keys is the world-1
  census.  This is what the one RCCL all-reduce per step sums over 8 GPUs.
* imcredist (src/imcredist.f:5-133) on the device: between steps every
  census packet is moved to rank 0 and then levelled with rebalance_plan,
  records travelling as packed device words (c2d_census_pack /
  c2d_census_append / c2d_census_truncate; between GPUs they go through RCCL
  send/recv, compton2d_amd/distributed.py).  Lineage keys make the histories
  independent of the tracking rank, so the summed tallies equal the
  single-rank oracle's.
"""
import numpy as np
import pytest
import torch

import oracle_lib as OL
from compton2d_amd import abi, distributed
from compton2d_amd.engine import Engine
from golden_io import GoldenCase

pytestmark = pytest.mark.gpu

TALLY_KEYS = ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in")
COUNTERS = [abi.CNT_STEPS, abi.CNT_ESCAPES, abi.CNT_CENSUS, abi.CNT_COLLIDE, abi.CNT_KILLED,
            abi.CNT_SOURCES, abi.CNT_COMPB, abi.CNT_EVENTS]


def _close(a, b, what):
    scale = max(np.max(np.abs(b)), 1e-300)
    np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-13 * scale, err_msg=what)


@pytest.mark.parametrize("name", ["ssc_tau", "c3_mrk421", "c2_32x32"])
def test_sharded_contexts_sum_to_world_one(name):
    gc = GoldenCase(name)
    steps = range(gc.nsteps)
    ref = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, device=0))
    want = []
    for n in steps:
        ref.transport_step(gc.step_inputs(n))
        want.append((ref.tallies(), set(ref.census()[2].tolist())))
    ref.close()
    for world in (2, 3):
        engs = [Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, device=0, rank=r, world=world))
                for r in range(world)]
        for n in steps:
            si = gc.step_inputs(n)
            parts, keys = [], []
            for e in engs:
                e.transport_step(si)
                parts.append(e.tallies())
                k = e.census()[2].tolist()
                keys += k
            t_ref, k_ref = want[n]
            cnt = sum(p["counters"] for p in parts)
            np.testing.assert_array_equal(cnt[COUNTERS], t_ref["counters"][COUNTERS],
                                          err_msg="%s world %d step %d" % (name, world, n))
            for k in TALLY_KEYS:
                _close(sum(np.asarray(p[k]) for p in parts), np.asarray(t_ref[k]),
                       "%s world %d step %d %s" % (name, world, n, k))
            assert len(keys) == len(set(keys)) == len(k_ref)
            assert set(keys) == k_ref
            # every rank tracked a share of the sources
            assert all(p["counters"][abi.CNT_SOURCES] > 0 for p in parts)
        for e in engs:
            e.close()


def _move(src, dst, first, n):
    """src's census records [first, first+n) -> appended to dst, through a
    device buffer (what RCCL send/recv carries between GPUs)."""
    if n == 0:
        return
    buf = torch.empty((n, abi.CENSUS_REC_WORDS), dtype=torch.int64, device="cuda:0")
    src.census_pack(first, n, buf.data_ptr())
    torch.cuda.synchronize()
    dst.census_append(buf.data_ptr(), n)


def test_device_census_rebalance_between_contexts_matches_oracle():
    gc = GoldenCase("ssc_tau")
    engs = [Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, device=0, rank=r, world=2,
                           census_capacity=1 << 20)) for r in range(2)]
    orc = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    for n in range(gc.nsteps):
        si = gc.step_inputs(n)
        parts = []
        for e in engs:
            e.transport_step(si)
            parts.append(e.tallies())
        assert orc.step(si) == 0
        to = orc.split()
        cnt = sum(p["counters"] for p in parts)
        np.testing.assert_array_equal(cnt[COUNTERS], to["counters"][COUNTERS])
        for k in TALLY_KEYS:
            _close(sum(np.asarray(p[k]) for p in parts), np.asarray(to[k]), "step %d %s" % (n, k))
        # skew: all census onto rank 0, then level with the plan every rank computes
        n1 = engs[1].census_count()
        _move(engs[1], engs[0], 0, n1)
        engs[1].census_truncate(0)
        counts = [e.census_count() for e in engs]
        plan = distributed.rebalance_plan(counts)
        assert plan == [(0, 1, counts[0] - (sum(counts) + 1) // 2)] or counts[0] <= 1
        for s, d, m in plan:
            keep = engs[s].census_count() - m
            _move(engs[s], engs[d], keep, m)
            engs[s].census_truncate(keep)
        c = [e.census_count() for e in engs]
        assert abs(c[0] - c[1]) <= 1 and sum(c) == len(orc.census()[2])
        keys = np.concatenate([e.census()[2] for e in engs])
        assert set(keys.tolist()) == set(orc.census()[2].tolist())
    for e in engs:
        e.close()
    orc.close()
