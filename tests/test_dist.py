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


def _workload_worker(rank, world, port, out):
    import sys
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as tdist

    import bench
    r, _, w = dist.init("gloo")
    res = {}
    for cfg in (2, 3, 4):
        wl = bench.workload(cfg, r, w, None)
        ids = torch.arange(wl["chain0"], wl["chain0"] + wl["C"])
        allids = [torch.zeros_like(ids) for _ in range(w)]
        tdist.all_gather(allids, ids)
        # dataset content per chain: residual checksum of each chain's dataset
        ck = torch.tensor([float(wl["ptas"][d].get_residuals()[0].sum()) for d in wl["ds"]],
                          dtype=torch.float64)
        ent = torch.tensor([wl["chain0"] // wl["per"] + int(d) for d in wl["ds"]])
        allent = [torch.zeros_like(ent) for _ in range(w)]
        tdist.all_gather(allent, ent)
        allck = [torch.zeros_like(ck) for _ in range(w)]
        tdist.all_gather(allck, ck)
        res[cfg] = (torch.cat(allids).tolist(), torch.cat(allck).tolist(), wl["C"],
                    torch.cat(allent).tolist())
    out.put((r, res))
    dist.finalize()


def test_two_rank_bench_workloads_partition_chains():
    """bench.py under torch.distributed.run: ranks own disjoint global chain ids (Philox
    keys) and agree on the data; config 4 shards the 256-dataset run_sims grid by dataset (strong scaling)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_workload_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for cfg in (2, 3, 4):
        ids, ck, C, _ = res[0][cfg]
        assert ids == res[1][cfg][0] and ck == res[1][cfg][1]   # both ranks see the same
        assert ids == list(range(2 * C))                        # disjoint, contiguous
    # configs 2/3: one dataset replicated on every rank; config 4: different datasets
    ck2 = res[0][2][1]
    assert len(set(ck2)) == 1
    ent4, C4 = res[0][4][3], res[0][4][2]
    assert set(ent4[:C4]).isdisjoint(set(ent4[C4:]))          # run_sims entries sharded
    assert sorted(set(ent4)) == list(range(256))              # 128 per rank, 64 chains each


def _gather_worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r, _, w = dist.init("gloo")
    got = dist.gather_chains(np.full((3, 2), float(r)) + np.arange(3)[:, None])
    out.put((r, None if got is None else got.tolist()))
    dist.finalize()


def test_gather_chains_goes_to_rank0_only():
    """The chain draws are gathered to rank 0 (the only consumer), not all-gathered."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    want = np.concatenate([np.full((3, 2), 0.0) + np.arange(3)[:, None],
                           np.full((3, 2), 1.0) + np.arange(3)[:, None]])
    assert np.array_equal(np.array(res[0]), want)
