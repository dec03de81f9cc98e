"""The multi-GPU tally exchange of bench.py's N > 1 path (bench.tally_exchange:
the id made by rank 0's c2d_comm_unique_id, broadcast with
torch.distributed, c2d_comm_init, c2d_allreduce_tallies on the library's
stream) inside a process that has torch and its own RCCL loaded, on the one
GPU a box has: a world of 1 (RCCL refuses two ranks on one device).  The
all-reduce of one rank is the identity, bit for bit; what this pins is that
the library's RCCL calls work next to torch's process group (the 8-GPU
driver run takes exactly this path)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_cabi_allreduce_beside_torch_process_group():
    import torch
    import torch.distributed as dist
    from compton2d_amd import abi
    from compton2d_amd.engine import Engine
    from golden_io import GoldenCase
    assert torch.cuda.is_available()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29631")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        gc = GoldenCase("ssc_tau")
        eng = Engine(gc.grid(comtot_mode=abi.COMTOT_TABLE, device=0))
        obj = [eng.comm_unique_id()]
        dist.broadcast_object_list(obj, src=0, device=torch.device("cuda", 0))
        eng.comm_init(obj[0], 0, 1)
        eng.transport_step(gc.step_inputs(0))
        before = eng.tallies_raw().copy()
        assert np.any(before != 0.0)
        eng.allreduce_tallies()
        np.testing.assert_array_equal(eng.tallies_raw(), before)
        # torch's own collective on the same device still works afterwards
        t = torch.ones(4, device="cuda:0")
        dist.all_reduce(t)
        assert float(t.sum()) == 4.0
        eng.close()
    finally:
        dist.destroy_process_group()
