"""bench.py's multi-GPU path on CPU: the --gpus N launcher, sharding and global diagnostics.

``--stub`` swaps the HIP sampler for a CPU AR(1) stand-in keyed by (seed, global chain id,
sweep) -- the same keying as the device Philox streams -- so a 2-rank run over gloo must
produce the same global R-hat / ESS as one process holding all the chains.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub",
                          "--steps", "6", "--warmup", "2", "--ess-burn", "4",
                          "--ess-window", "60", *args], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_two_rank_launch_matches_one_process():
    two = _run("--gpus", "2", "--chains", "6")
    one = _run("--gpus", "1", "--chains", "12")
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["chains_total"] == one["config"]["chains_total"] == 12
    assert two["shards"] == [[0, 6], [6, 12]] and one["shards"] == [[0, 12]]
    # global diagnostics over ALL chains: identical draws -> identical R-hat and ESS
    w2, w1 = two["ess_window"], one["ess_window"]
    assert w2["chains"] == w1["chains"] == 12
    for k in w1["rhat_max"]:
        assert w2["rhat_max"][k] == w1["rhat_max"][k]
        assert w2["ess_total"][k] == w1["ess_total"][k]
    assert two["cpu_baseline"] is None


def test_launcher_reports_world_size_four():
    four = _run("--gpus", "4", "--chains", "3")
    assert four["n_gpus"] == 4 and four["config"]["chains_total"] == 12
    assert [s[0] for s in four["shards"]] == [0, 3, 6, 9]


def test_launcher_fails_fast_when_a_rank_dies():
    """One rank exits 3 right after init while its peers wait in a collective: the launcher
    must return non-zero within seconds and leave no rank process behind."""
    import time
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub",
                          "--gpus", "3", "--chains", "4", "--steps", "4", "--warmup", "1",
                          "--ess-burn", "2", "--ess-window", "20", "--stub-fail-rank", "1"],
                         env=env, capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert took < 60, took
    pids = [int(p) for ln in out.stderr.splitlines() if ln.startswith("bench launcher: rank pids")
            for p in ln.split()[4:]]
    assert len(pids) == 3
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, f"rank process {pid} left running"


def test_global_diagnostics_converged_datasets_per_model():
    """bench.global_diagnostics with run_sims groups: per model, the ESS of the datasets whose
    every split R-hat <= 1.01 (config 4's ess_by_model[...]['converged_datasets'])."""
    import numpy as np

    import bench
    rng = np.random.default_rng(0)
    C, S = 16, 400
    dsid = np.repeat(np.arange(4), C)
    draws = rng.normal(size=(4 * C, S, 2))
    draws[dsid == 3, :, 0] += np.where(np.arange(C) < C // 2, 5.0, 0.0)[:, None]  # bimodal
    theta = rng.uniform(size=(4 * C, S))
    groups = np.array(["a", "a", "b", "b"])
    ess, rhat, by, conv = bench.global_diagnostics(draws, theta, dsid, ["p0", "p1"],
                                                   np.array([True] * 4), groups)
    assert conv["a"][1:] == [2, 2] and conv["b"][1:] == [1, 2]
    assert by["b"][1]["p0"] > 1.5 and max(by["a"][1].values()) <= 1.01
    # the converged datasets' ESS is the per-dataset ESS summed over them
    assert 0 < conv["b"][0]["p0"] < by["b"][0]["p0"]
