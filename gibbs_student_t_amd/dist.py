"""Multi-GPU sharding of independent chains (one process per GPU, torch.distributed).

Chains never exchange data while sampling: rank r owns global chains
[r*C, (r+1)*C) and keys its Philox streams by global chain id, so a sharded run equals a
single-GPU run chain for chain.  The only collectives are the final reductions of chain
summaries (ESS sums, R-hat maxima, timing maxima) -- RCCL over xGMI with backend "nccl",
gloo on CPU.
"""
from __future__ import annotations

import datetime
import os

import numpy as np

# Finite collective timeout: a rank that dies leaves its peers blocked in a collective;
# with a finite timeout they fail instead of holding the GPUs until the box's own limit.
DEFAULT_TIMEOUT_S = float(os.environ.get("GST_DIST_TIMEOUT_S", "300"))


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str | None = None):
    """Initialise the process group when launched by torch.distributed.run.  The backend is
    RCCL ("nccl") with a GPU, gloo without; ``GST_DIST_BACKEND`` overrides it (gloo ranks
    sharing one GPU rehearse the multi-rank path on a one-GPU box: RCCL refuses two ranks
    on one device)."""
    import torch.distributed as dist
    rank, local, world = env_rank()
    if world <= 1 or dist.is_initialized():
        return rank, local, world
    backend = os.environ.get("GST_DIST_BACKEND") or backend
    if backend is None:
        import torch
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=DEFAULT_TIMEOUT_S))
    return rank, local, world


def chain_range(rank: int, chains_per_rank: int):
    """Global chain ids owned by ``rank`` (weak scaling: fixed chains per GPU)."""
    return rank * chains_per_rank, (rank + 1) * chains_per_rank


def _coll_device(device):
    """Where a collective's tensors live: the rank's GPU under RCCL, host memory otherwise."""
    import torch
    import torch.distributed as dist
    if device is not None and dist.get_backend() == "nccl":
        return device
    return torch.device("cpu")


def reduce_summary(vec_sum: np.ndarray, vec_max: np.ndarray, device=None):
    """All-reduce per-rank summaries: sums (ESS, counts) and maxima (time, R-hat)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return np.asarray(vec_sum, float), np.asarray(vec_max, float)
    dev = _coll_device(device)
    s = torch.as_tensor(np.asarray(vec_sum, float), device=dev)
    m = torch.as_tensor(np.asarray(vec_max, float), device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return s.cpu().numpy(), m.cpu().numpy()


def gather_chains(arr: np.ndarray, device=None):
    """Gather per-chain arrays (leading axis = this rank's chains, same shape on every
    rank) to rank 0, in rank order, i.e. global chain order: the one data collective of a
    run, so R-hat / ESS are computed over ALL chains, not per rank.  Only
    rank 0 uses the draws, so only rank 0 receives them (a gather, not an all-gather): one
    ~C x draws x params fp64 block per rank over RCCL (xGMI) on GPU ranks, once per run.
    Returns the gathered array on rank 0 and None on the other ranks."""
    import torch
    import torch.distributed as dist
    a = np.ascontiguousarray(arr, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return a
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = _coll_device(device)
    t = torch.as_tensor(a, device=dev)
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=parts, dst=0)
    if rank != 0:
        return None
    return torch.cat(parts, dim=0).cpu().numpy()


def barrier(device=None):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        if device is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def finalize():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
