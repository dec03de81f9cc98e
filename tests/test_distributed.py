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
