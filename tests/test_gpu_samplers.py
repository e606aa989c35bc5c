"""The kernel's own Gamma / Beta samplers on MI355X, through gst_debug_variates (ABI 6).

The injected-variate parity tests feed Gamma and Beta *values* from the reference's tape
(parity contract 3), so the Philox samplers themselves are checked here, by
distribution:

* gamma_mt (Marsaglia-Tsang, a < 1 by the a + 1 boost; the theta stage) and gamma_mt_slots<4>
  (the alpha stage's interleaved copy, gibbs.py:239) for shapes 0.5 - 2 -- the lower tail
  P(G < eps) for eps = 1e-2 ... 1e-8 on ~1e8 draws against scipy.stats.gamma.cdf (binomial
  z-scores), which sets alpha = (nu / 2) / G of every z = 0 TOA when nu ~ 1-2, and the
  bulk by a KS test on 2e6 draws;
* the theta Beta (two gamma_mt draws, gibbs.py:196) at the shapes the ecq / J1713 posteriors
  give it, KS against scipy.stats.beta and its mean within 5 standard errors.
"""
import numpy as np
import pytest
import scipy.stats

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

EPS = (1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-8)
CHUNK = 1 << 23                # a multiple of 256 (gamma_slots draws 4 x 64 per wave)
NTAIL = 12 * CHUNK             # ~1e8 draws


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _tail_counts(kind, a, seed):
    from gibbs_student_t_amd.native import debug_variates
    eps = torch.tensor(EPS, dtype=torch.float64, device="cuda:0")
    cnt = torch.zeros(len(EPS), dtype=torch.float64, device="cuda:0")
    for call in range(NTAIL // CHUNK):
        g = debug_variates(kind, a, CHUNK, seed=seed, call=call)
        assert bool(torch.all(torch.isfinite(g) & (g > 0))), "non-finite or non-positive draw"
        cnt += (g[None, :] < eps[:, None]).sum(dim=1).to(torch.float64)
        del g
    return cnt.cpu().numpy()


@pytest.mark.parametrize("kind", ["gamma", "gamma_slots"])
@pytest.mark.parametrize("a", [0.5, 0.7, 1.0, 1.5])
def test_gamma_lower_tail(kind, a):
    """P(G < eps) on ~1e8 draws: every eps within 5 binomial standard deviations of the exact
    probability (which runs from ~0.08 down to 2e-5 .. 1e-8 over the shapes)."""
    cnt = _tail_counts(kind, a, seed=1000 + int(10 * a))
    p = scipy.stats.gamma.cdf(np.array(EPS), a)
    sd = np.sqrt(NTAIL * p * (1 - p))
    z = (cnt - NTAIL * p) / np.maximum(sd, 1.0)
    # where fewer than ~25 draws are expected the binomial is Poisson: |count - mean| <= 5 sd + 3
    ok = np.abs(cnt - NTAIL * p) <= 5 * sd + 3
    assert ok.all(), {f"{e:g}": (int(c), float(NTAIL * q), float(zz))
                      for e, c, q, zz in zip(EPS, cnt, p, z)}


@pytest.mark.parametrize("kind", ["gamma", "gamma_slots"])
@pytest.mark.parametrize("a", [0.5, 0.7, 1.0, 2.0, 40.0])
def test_gamma_bulk(kind, a):
    from gibbs_student_t_amd.native import debug_variates
    g = debug_variates(kind, a, 1 << 21, seed=77, call=int(10 * a)).cpu().numpy()
    p = scipy.stats.kstest(g, scipy.stats.gamma(a).cdf).pvalue
    assert p > 1e-3, (kind, a, p)
    se = np.sqrt(a / len(g))
    assert abs(g.mean() - a) < 5 * se, (g.mean(), a)


@pytest.mark.parametrize("a,b", [(2.72, 141.28), (4.72, 139.28), (1.3, 72.0), (8.0, 8.0)])
def test_theta_beta(a, b):
    """Beta(sum z + n m, n - sum z + n (1 - m)) as the theta stage draws it: J1713 (n = 130,
    m = 0.01) with 2 / 4 flagged TOAs, ecq-like shapes, and a symmetric case."""
    from gibbs_student_t_amd.native import debug_variates
    x = debug_variates("beta", a, 2_000_000, b=b, seed=5, call=int(a * 100)).cpu().numpy()
    p = scipy.stats.kstest(x, scipy.stats.beta(a, b).cdf).pvalue
    assert p > 1e-3, (a, b, p)
    mean, var = a / (a + b), a * b / ((a + b) ** 2 * (a + b + 1))
    assert abs(x.mean() - mean) < 5 * np.sqrt(var / len(x)), (x.mean(), mean)
