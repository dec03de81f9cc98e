"""One process per GPU; the per-step tally exchange over RCCL.

The reference sums its per-worker tallies with thousands of scalar
MPI_REDUCE calls every step (src/xec2d.f:325-399 xec_add / graphics_collect,
src/update2d.f:1929-2078 cens_add_up / E_add_up).  Here the sources of a step
are sharded by lineage index (global source index % world == rank, see
compton2d_amd/csrc/transport.hip) with no data-path exchange, and the fused
f64 tally buffer (include/compton2d.h c2d_tally_layout) is summed with ONE
all-reduce: backend "nccl" (= RCCL over xGMI) on MI355X, "gloo" on CPU.
"""
from __future__ import annotations

import os


def env_rank():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init(backend: str | None = None):
    """Initialise torch.distributed from the torchrun environment (world > 1)."""
    rank, world, local = env_rank()
    if world > 1:
        import torch
        import torch.distributed as dist
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {}
            if backend == "nccl":
                kw["device_id"] = torch.device("cuda", local)
            dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def is_dist() -> bool:
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    except Exception:
        return False


def allreduce_tallies(tensor) -> None:
    """Sum the fused tally buffer over all ranks in place (no-op for one rank)."""
    if is_dist():
        import torch.distributed as dist
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM)


def allreduce_max(value: float, device=None) -> float:
    if not is_dist():
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None) -> None:
    if is_dist():
        import torch.distributed as dist
        if device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
