"""Multi-GPU sharding of independent chains (one process per GPU, torch.distributed).

Chains never exchange data while sampling: rank r owns global chains
[r*C, (r+1)*C) and keys its Philox streams by global chain id, so a sharded run equals a
single-GPU run chain for chain.  The only collectives are the final reductions of chain
summaries (ESS sums, R-hat maxima, timing maxima) -- RCCL over xGMI with backend "nccl",
gloo on CPU.
"""
from __future__ import annotations

import os

import numpy as np


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str | None = None):
    """Initialise the process group when launched by torch.distributed.run."""
    import torch.distributed as dist
    rank, local, world = env_rank()
    if world <= 1 or dist.is_initialized():
        return rank, local, world
    if backend is None:
        import torch
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, local, world


def chain_range(rank: int, chains_per_rank: int):
    """Global chain ids owned by ``rank`` (weak scaling: fixed chains per GPU)."""
    return rank * chains_per_rank, (rank + 1) * chains_per_rank


def reduce_summary(vec_sum: np.ndarray, vec_max: np.ndarray, device=None):
    """All-reduce per-rank summaries: sums (ESS, counts) and maxima (time, R-hat)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return np.asarray(vec_sum, float), np.asarray(vec_max, float)
    dev = device if device is not None else torch.device("cpu")
    s = torch.as_tensor(np.asarray(vec_sum, float), device=dev)
    m = torch.as_tensor(np.asarray(vec_max, float), device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return s.cpu().numpy(), m.cpu().numpy()


def gather_chains(arr: np.ndarray, device=None) -> np.ndarray:
    """All-gather per-chain arrays (leading axis = this rank's chains, same shape on
    every rank) in rank order, i.e. global chain order: the one data collective of a run
    (SURVEY.md 8e), so R-hat / ESS are computed over ALL chains, not per rank.  On GPU
    ranks the tensors travel over RCCL (xGMI); one ~C x draws x params fp64 block per rank,
    once per run."""
    import torch
    import torch.distributed as dist
    a = np.ascontiguousarray(arr, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return a
    world = dist.get_world_size()
    dev = device if device is not None else torch.device("cpu")
    t = torch.as_tensor(a, device=dev)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    dist.all_gather_into_tensor(out, t)
    return out.cpu().numpy()


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
