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
    """(rank, world, local device) from the torchrun environment.  Rehearsal
    on a one-GPU box: C2D_ONE_GPU=1 puts every rank on device 0 (with
    C2D_DIST_BACKEND=gloo, since RCCL refuses two ranks on one device)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("C2D_ONE_GPU") == "1":
        local = 0
    return rank, world, local


def init(backend: str | None = None):
    """Initialise torch.distributed from the torchrun environment (world > 1)."""
    rank, world, local = env_rank()
    if world > 1:
        import torch
        import torch.distributed as dist
        if not dist.is_initialized():
            if backend is None:
                backend = os.environ.get("C2D_DIST_BACKEND") or (
                    "nccl" if torch.cuda.is_available() else "gloo")
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
    """Sum the fused tally buffer over all ranks in place (no-op for one rank).

    The reduction is ordered on torch's stream only, while the engine reads
    the tallies (n_field, ecens for c2d_fp_step) on its own non-blocking HIP
    stream: wait for it here so the engine never sees un-reduced tallies."""
    if is_dist():
        import torch
        import torch.distributed as dist
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM)
        if tensor.is_cuda:
            torch.cuda.synchronize(tensor.device)


def allreduce_max(value: float, device=None) -> float:
    if not is_dist():
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(value: float, device=None) -> float:
    if not is_dist():
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier(device=None) -> None:
    if is_dist():
        import torch.distributed as dist
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


# ---------------------------------------------------------------------------
# census load balance (replaces imcredist, src/imcredist.f:5-133)
# ---------------------------------------------------------------------------
REC_WORDS = 13   # 6 f64 + 5 i32 + lineage key as two 32-bit halves, all exact in f64


def rebalance_plan(counts):
    """Deterministic moves (src, dst, n) that level `counts` to
    total//W (+1 on the lowest ranks): surplus ranks, in rank order, fill
    deficit ranks in rank order (every rank computes the same plan)."""
    W = len(counts)
    total = int(sum(counts))
    target = [total // W + (1 if r < total % W else 0) for r in range(W)]
    sur = [[r, int(counts[r]) - target[r]] for r in range(W) if counts[r] > target[r]]
    dfc = [[r, target[r] - int(counts[r])] for r in range(W) if counts[r] < target[r]]
    plan, i, j = [], 0, 0
    while i < len(sur) and j < len(dfc):
        n = min(sur[i][1], dfc[j][1])
        plan.append((sur[i][0], dfc[j][0], n))
        sur[i][1] -= n
        dfc[j][1] -= n
        if sur[i][1] == 0:
            i += 1
        if dfc[j][1] == 0:
            j += 1
    return plan


def _pack(d6, i5, keys):
    import numpy as np
    k = np.asarray(keys, np.uint64)
    return np.column_stack([np.asarray(d6, np.float64), np.asarray(i5, np.float64),
                            (k & np.uint64(0xFFFFFFFF)).astype(np.float64),
                            (k >> np.uint64(32)).astype(np.float64)])


def _unpack(rec):
    import numpy as np
    rec = np.asarray(rec, np.float64).reshape(-1, REC_WORDS)
    keys = rec[:, 11].astype(np.uint64) | (rec[:, 12].astype(np.uint64) << np.uint64(32))
    return rec[:, :6].copy(), rec[:, 6:11].astype(np.int32), keys


def _comm_device(device):
    """Tensors for the collectives live where the backend needs them: the
    rank's GPU for nccl (RCCL), the host for gloo."""
    if device is not None:
        return device
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return torch.device("cpu")


def rebalance_census(d6, i5, keys, device=None):
    """Level the census record counts over the ranks (records as exported by
    Engine.census(): d6 [n,6], i5 [n,5], keys [n]).  Records move whole, so
    with lineage keys the histories, and every tally, do not depend on which
    rank tracks them.  Collectives: one all_gather of the counts, then
    point-to-point transfers of the surplus records."""
    import numpy as np
    if not is_dist():
        return d6, i5, keys
    import torch
    import torch.distributed as dist
    rank, W = dist.get_rank(), dist.get_world_size()
    device = _comm_device(device)
    n = len(keys)
    cnt = torch.tensor([n], dtype=torch.int64, device=device)
    allc = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(W)]
    dist.all_gather(allc, cnt)
    counts = [int(c.item()) for c in allc]
    plan = rebalance_plan(counts)
    rec = _pack(d6, i5, keys)
    keep = n - sum(m for s, _, m in plan if s == rank)
    ops, sends, recvs = [], [], []
    off = keep
    for s, d, m in plan:
        if s == rank:
            t = torch.from_numpy(np.ascontiguousarray(rec[off:off + m])).to(device)
            off += m
            sends.append(t)
            ops.append(dist.P2POp(dist.isend, t, d))
        elif d == rank:
            t = torch.empty((m, REC_WORDS), dtype=torch.float64, device=device)
            recvs.append(t)
            ops.append(dist.P2POp(dist.irecv, t, s))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    parts = [rec[:keep]] + [t.cpu().numpy() for t in recvs]
    return _unpack(np.concatenate(parts) if parts else rec[:0])


def rebalance_engine_census(engine, threshold: float = 0.1, device=None, packed=None) -> bool:
    """imcredist for an Engine: when the largest census exceeds the mean by
    more than `threshold`, level the census counts (all ranks call it).  On
    the nccl backend (RCCL) the records never leave the GPUs: the surplus tail
    is packed on the device (c2d_census_pack), sent with RCCL send/recv and
    appended on the receiving GPU (c2d_census_append); on gloo they go
    through the host (export / import).  `packed` forces either path (the
    packed one on host tensors: the CPU tests drive it with gloo)."""
    if not is_dist():
        return False
    import torch
    import torch.distributed as dist
    device = _comm_device(device)
    n = engine.census_count()
    t = torch.tensor([float(n)], dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    mean = float(t.item()) / dist.get_world_size()
    if mean <= 0 or float(mx.item()) <= (1.0 + threshold) * mean:
        return False
    if packed is None:
        packed = device.type == "cuda"
    if packed:
        _rebalance_device(engine, device)
    else:
        d6, i5, keys = engine.census()
        engine.import_census(*rebalance_census(d6, i5, keys, device=device))
    return True


def _rebalance_device(engine, device) -> None:
    """Level the census over the ranks with packed device records and RCCL
    point-to-point transfers (replaces imcredist's master-relayed MPI copies,
    src/imcredist.f:18-123)."""
    import torch
    import torch.distributed as dist
    from . import abi
    rank, W = dist.get_rank(), dist.get_world_size()
    n = engine.census_count()
    cnt = torch.tensor([n], dtype=torch.int64, device=device)
    allc = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(W)]
    dist.all_gather(allc, cnt)
    plan = rebalance_plan([int(c.item()) for c in allc])
    keep = n - sum(m for s, _, m in plan if s == rank)
    ops, recvs, off = [], [], keep
    for s, d, m in plan:
        if s == rank:
            t = torch.empty((m, abi.CENSUS_REC_WORDS), dtype=torch.int64, device=device)
            engine.census_pack(off, m, t.data_ptr())        # synchronous on the engine's stream
            off += m
            ops.append(dist.P2POp(dist.isend, t, d))
        elif d == rank:
            t = torch.empty((m, abi.CENSUS_REC_WORDS), dtype=torch.int64, device=device)
            recvs.append(t)
            ops.append(dist.P2POp(dist.irecv, t, s))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    engine.census_truncate(keep)
    for t in recvs:
        engine.census_append(t.data_ptr(), t.shape[0])
