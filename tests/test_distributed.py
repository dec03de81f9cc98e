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
