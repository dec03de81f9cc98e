"""Multi-rank path on CPU (gloo, world_size 2): lineage-sharded sources +
one all-reduce of the fused tally buffer reproduce the single-rank result.

Each rank runs the oracle in lineage mode with rank/world sharding — the same
(global source index % world == rank) rule the HIP kernel applies — and sums
its tallies with compton2d_amd.distributed.allreduce_tallies, the function
bench.py uses over RCCL on MI355X.  Census packets stay on the rank that made
them (no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as OL
from compton2d_amd import abi, distributed
from golden_io import GoldenCase


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, nsteps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    distributed.init(backend="gloo")
    gc = GoldenCase(name)
    o = OL.Oracle(gc.grid(rank=rank, world=world), OL.RNG_LINEAGE, "det")
    out = []
    for n in range(nsteps):
        assert o.step(gc.step_inputs(n)) == 0
        t = torch.from_numpy(o.tallies())
        distributed.allreduce_tallies(t)
        ncens = torch.tensor([float(o.lib.c2o_census_count(o.ctx))], dtype=torch.float64)
        distributed.allreduce_tallies(ncens)
        out.append((t.numpy().copy(), float(ncens.item())))
    if rank == 0:
        q.put(out)
    distributed.barrier()
    dist.destroy_process_group()
    o.close()


@pytest.mark.parametrize("name", ["ssc_tau", "ec_lower"])
def test_two_rank_gloo_equals_single_rank(name):
    nsteps = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, nsteps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    gc = GoldenCase(name)
    o = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    L = abi.tally_layout(gc.nz, gc.nr, gc.nmu)
    c0 = L["counters"][0]
    for n in range(nsteps):
        assert o.step(gc.step_inputs(n)) == 0
        ref = o.tallies()
        t, ncens = got[n]
        np.testing.assert_array_equal(t[c0:c0 + 8], ref[c0:c0 + 8])      # integer counters
        np.testing.assert_allclose(t, ref, rtol=1e-11, atol=1e-13 * np.abs(ref).max())
        assert ncens == o.lib.c2o_census_count(o.ctx)
    o.close()


# ---------------------------------------------------------------------------
# census rebalance (imcredist, src/imcredist.f:5-133)
# ---------------------------------------------------------------------------
def test_rebalance_plan_levels_counts():
    for counts in ([1000, 10], [5, 5, 30, 0], [3, 3, 3], [0, 0, 7], [9, 0, 0, 0, 1]):
        plan = distributed.rebalance_plan(counts)
        c = list(counts)
        for s, d, m in plan:
            assert m > 0 and s != d
            c[s] -= m
            c[d] += m
        assert max(c) - min(c) <= 1 and sum(c) == sum(counts)


def _rebalance_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    distributed.init(backend="gloo")
    rng = np.random.default_rng(rank)
    n = 1000 if rank == 0 else 10
    d6 = rng.normal(size=(n, 6))
    i5 = rng.integers(0, 200, (n, 5)).astype(np.int32)
    keys = rng.integers(0, 2 ** 63, n, dtype=np.uint64) | np.uint64(rank)
    out = distributed.rebalance_census(d6, i5, keys)
    q.put((rank, (d6, i5, keys), out))
    distributed.barrier()
    dist.destroy_process_group()


def test_rebalance_census_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rebalance_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    before = {int(k): (tuple(d), tuple(i)) for r in res for d, i, k in zip(*res[r][0])}
    after = {}
    for r in res:
        d6, i5, keys = res[r][1]
        assert len(keys) == 505
        after.update({int(k): (tuple(d), tuple(i)) for d, i, k in zip(d6, i5, keys)})
    assert after == before          # every record arrives whole, exactly once


def _skew_to_rank0(d6, i5, keys):
    """Move every census record to rank 0 (a worst-case imbalance)."""
    rank = dist.get_rank()
    n = torch.tensor([len(keys)], dtype=torch.int64)
    allc = [torch.zeros(1, dtype=torch.int64) for _ in range(dist.get_world_size())]
    dist.all_gather(allc, n)
    if rank == 0:
        parts = [distributed._pack(d6, i5, keys)]
        for r in range(1, len(allc)):
            t = torch.empty((int(allc[r].item()), distributed.REC_WORDS), dtype=torch.float64)
            dist.recv(t, r)
            parts.append(t.numpy())
        return distributed._unpack(np.concatenate(parts))
    dist.send(torch.from_numpy(distributed._pack(d6, i5, keys)), 0)
    return distributed._unpack(np.zeros((0, distributed.REC_WORDS)))


def _rebalanced_run_worker(rank, world, port, name, nsteps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    distributed.init(backend="gloo")
    gc = GoldenCase(name)
    o = OL.Oracle(gc.grid(rank=rank, world=world), OL.RNG_LINEAGE, "det")
    out = []
    for n in range(nsteps):
        assert o.step(gc.step_inputs(n)) == 0
        t = torch.from_numpy(o.tallies())
        distributed.allreduce_tallies(t)
        out.append(t.numpy().copy())
        d6, i5, keys = _skew_to_rank0(*o.census())   # all census on rank 0 ...
        o.import_census(*distributed.rebalance_census(d6, i5, keys))   # ... then levelled
    if rank == 0:
        q.put(out)
    distributed.barrier()
    dist.destroy_process_group()
    o.close()


def test_rebalanced_census_leaves_tallies_unchanged():
    """Lineage-keyed histories: moving census packets between ranks between
    steps gives the single-rank tallies (to summation order)."""
    name, nsteps = "ssc_tau", 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rebalanced_run_worker, args=(r, 2, port, name, nsteps, q))
             for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    gc = GoldenCase(name)
    o = OL.Oracle(gc.grid(), OL.RNG_LINEAGE, "det")
    L = abi.tally_layout(gc.nz, gc.nr, gc.nmu)
    c0 = L["counters"][0]
    for n in range(nsteps):
        assert o.step(gc.step_inputs(n)) == 0
        ref = o.tallies()
        np.testing.assert_array_equal(got[n][c0:c0 + 8], ref[c0:c0 + 8])
        np.testing.assert_allclose(got[n], ref, rtol=1e-11, atol=1e-13 * np.abs(ref).max())
    o.close()


# ---------------------------------------------------------------------------
# rebalance_engine_census (imcredist for an Engine, src/imcredist.f:18-123),
# the call an N > 1 run makes, on gloo world 2 with a census skewed first to
# rank 0 and then to rank 1, so records move in both directions
# ---------------------------------------------------------------------------
class _OracleEngine:
    """The Engine census interface (census_count / census / import_census)
    over an oracle context: rebalance_engine_census's export/import path."""

    def __init__(self, o):
        self.o = o

    def census_count(self):
        return int(self.o.lib.c2o_census_count(self.o.ctx))

    def census(self):
        return self.o.census()

    def import_census(self, d6, i5, keys):
        assert self.o.import_census(d6, i5, keys) == 0


class _PackedEngine:
    """The Engine's packed-record interface (census_count / census_pack /
    census_append / census_truncate on c2d_census_pack's 8-word records,
    abi.CENSUS_REC_WORDS) over a host array: the device path's plan,
    offsets, truncation and append order, driven with host tensors."""

    def __init__(self, rec):
        self.rec = np.array(rec, np.int64).reshape(-1, abi.CENSUS_REC_WORDS)

    def census_count(self):
        return len(self.rec)

    def census_pack(self, off, m, ptr):
        import ctypes
        assert 0 <= off and off + m <= len(self.rec)
        ctypes.memmove(ptr, self.rec[off:off + m].ctypes.data, m * abi.CENSUS_REC_WORDS * 8)

    def census_truncate(self, keep):
        assert 0 <= keep <= len(self.rec)
        self.rec = self.rec[:keep]

    def census_append(self, ptr, m):
        import ctypes
        add = np.empty((m, abi.CENSUS_REC_WORDS), np.int64)
        ctypes.memmove(add.ctypes.data, ptr, m * abi.CENSUS_REC_WORDS * 8)
        self.rec = np.concatenate([self.rec, add])


def _engine_rebalance_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    distributed.init(backend="gloo")
    out = {}
    # export/import path: the oracle's own census after a step of ssc_tau
    # (the ranks' lineage shards), skewed to rank 0, levelled, then the
    # surplus of a second step skewed to rank 1, levelled again
    gc = GoldenCase("ssc_tau")
    o = OL.Oracle(gc.grid(rank=rank, world=world), OL.RNG_LINEAGE, "det")
    assert o.step(gc.step_inputs(0)) == 0
    eng = _OracleEngine(o)
    d6, i5, keys = _skew_to_rank0(*o.census())
    eng.import_census(d6, i5, keys)
    before = eng.census()
    moved0 = distributed.rebalance_engine_census(eng, packed=False)
    after0 = eng.census()
    d6, i5, keys = eng.census()
    if rank == 1:     # rank 1 takes a copy of rank 0's records under fresh keys
        extra = 3 * len(keys)
        d6 = np.concatenate([d6] + [d6] * 3)
        i5 = np.concatenate([i5] + [i5] * 3)
        keys = np.concatenate([keys] + [keys + np.uint64((i + 1) << 40) for i in range(3)])
        assert len(keys) == 4 * len(after0[2]) and extra > 0
    eng.import_census(d6, i5, keys)
    mid = eng.census()
    moved1 = distributed.rebalance_engine_census(eng, packed=False)
    after1 = eng.census()
    out["oracle"] = (before, after0, mid, after1, moved0, moved1)
    o.close()
    # packed path: 8-word records, 900 on rank 0 / 100 on rank 1, then 50 / 2000
    rng = np.random.default_rng(7 + rank)
    pe = _PackedEngine(rng.integers(-2 ** 62, 2 ** 62, (900 if rank == 0 else 100, abi.CENSUS_REC_WORDS)))
    p_before = pe.rec.copy()
    pm0 = distributed.rebalance_engine_census(pe, packed=True)
    p_after0 = pe.rec.copy()
    pe.rec = rng.integers(-2 ** 62, 2 ** 62, (50 if rank == 0 else 2000, abi.CENSUS_REC_WORDS))
    p_mid = pe.rec.copy()
    pm1 = distributed.rebalance_engine_census(pe, packed=True)
    out["packed"] = (p_before, p_after0, p_mid, pe.rec.copy(), pm0, pm1)
    q.put((rank, out))
    distributed.barrier()
    dist.destroy_process_group()


def _records(cens):
    d6, i5, keys = cens
    return sorted((int(k), tuple(d), tuple(i)) for d, i, k in zip(d6, i5, keys))


def test_rebalance_engine_census_both_directions_gloo():
    """rebalance_engine_census on 2 gloo ranks: a census skewed to rank 0 is
    levelled (0 -> 1), then one skewed to rank 1 (1 -> 0), through both
    paths -- export/import (oracle census records) and the packed-record
    path of the nccl backend (census_pack / truncate / append, here on host
    tensors).  Every record arrives whole, exactly once, and the counts end
    level; the rank that keeps records keeps its first ones in order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_rebalance_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    # export / import
    b = {r: res[r]["oracle"] for r in (0, 1)}
    assert all(b[r][4] and b[r][5] for r in (0, 1))          # both calls moved records
    assert len(b[1][0][2]) == 0 < len(b[0][0][2])            # first skew: all on rank 0
    assert len(b[1][2][2]) > len(b[0][2][2])                 # second skew: rank 1 heavier
    for phase_in, phase_out in ((0, 1), (2, 3)):
        assert _records(tuple(np.concatenate([b[r][phase_in][i] for r in (0, 1)]) for i in range(3))) == \
            _records(tuple(np.concatenate([b[r][phase_out][i] for r in (0, 1)]) for i in range(3)))
        n0, n1 = len(b[0][phase_out][2]), len(b[1][phase_out][2])
        assert abs(n0 - n1) <= 1
    # packed records
    p = {r: res[r]["packed"] for r in (0, 1)}
    assert all(p[r][4] and p[r][5] for r in (0, 1))
    for phase_in, phase_out, keeper in ((0, 1, 1), (2, 3, 0)):
        before = np.concatenate([p[0][phase_in], p[1][phase_in]])
        after = np.concatenate([p[0][phase_out], p[1][phase_out]])
        assert sorted(map(tuple, before)) == sorted(map(tuple, after))
        assert len(p[0][phase_out]) == len(p[1][phase_out]) == len(before) // 2
        # the deficit rank keeps its own records first, the surplus rank its head
        np.testing.assert_array_equal(p[keeper][phase_out][:len(p[keeper][phase_in])], p[keeper][phase_in])
        donor = 1 - keeper
        np.testing.assert_array_equal(p[donor][phase_out], p[donor][phase_in][:len(p[donor][phase_out])])
