"""bench.py's multi-rank path with the HIP sampler, rehearsed on one GPU.

RCCL refuses two ranks on one device, so the ranks talk over gloo (GST_DIST_BACKEND) and
share the box's GPU; everything else is the production path: the --gpus N launcher, chain
sharding by global id (rank r owns chains [r C, (r+1) C)), the gather of every chain's
window draws to rank 0, global R-hat / ESS and the max-over-ranks timing.  Chains are keyed
by global id, so two ranks of C chains must give rank 0 exactly the draws of one rank with
2 C chains: identical R-hat and ESS, bit for bit.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = dict(os.environ, GST_DIST_BACKEND="gloo")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"),
                          "--steps", "8", "--warmup", "2", "--ess-burn", "20",
                          "--ess-window", "100", "--no-cpu-baseline", "--no-stage-costs", *args],
                         env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_two_ranks_equal_one_rank_with_all_chains():
    pytest.importorskip("torch")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    two = _bench("--gpus", "2", "--chains", "128")
    one = _bench("--gpus", "1", "--chains", "256")
    assert two["n_gpus"] == 2 and two["shards"] == [[0, 128], [128, 256]]
    assert one["config"]["chains_total"] == two["config"]["chains_total"] == 256
    assert two["chains_with_status"] == one["chains_with_status"] == 0
    assert two["value"] > 0 and two["kernel_ms"] > 0
    w2, w1 = two["ess_window"], one["ess_window"]
    assert w2["chains"] == w1["chains"] == 256
    for k in w1["rhat_max"]:
        assert w2["rhat_max"][k] == w1["rhat_max"][k], k
        assert w2["ess_total"][k] == w1["ess_total"][k], k
