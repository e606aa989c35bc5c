"""Chain sharding and the final summary all-reduce, world_size 2 over gloo (CPU)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gibbs_student_t_amd import dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r, _, w = dist.init("gloo")
    lo, hi = dist.chain_range(r, 8)
    s, m = dist.reduce_summary(np.array([float(hi - lo), 10.0 * r]),
                               np.array([1.0 + r, -float(r)]))
    dist.barrier()
    out.put((r, lo, hi, s.tolist(), m.tolist()))
    dist.finalize()


def test_two_rank_summary_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, s0, m0), (r1, lo1, hi1, s1, m1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 8, 8, 16)       # disjoint global chain ids
    assert s0 == s1 == [16.0, 10.0]                     # summed over ranks
    assert m0 == m1 == [2.0, 0.0]                       # max over ranks


def test_single_process_is_identity():
    s, m = dist.reduce_summary(np.array([1.0, 2.0]), np.array([3.0]))
    assert s.tolist() == [1.0, 2.0] and m.tolist() == [3.0]
    assert dist.chain_range(3, 1024) == (3072, 4096)
