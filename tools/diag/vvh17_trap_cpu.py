"""CPU experiment: how fast vvh17 chains leave the all-outlier start (z = 1, alpha = 1e10).

    OPENBLAS_NUM_THREADS=1 python tools/diag/vvh17_trap_cpu.py svd|chol SEED

Runs the oracle (bit-exact to gibbs.py with the legacy RNG) from a prior draw and prints
sum(z) every 100 sweeps.  ``svd`` is the reference's b draw (gibbs.py:169-180); ``chol``
replaces only the draw by the exact Cholesky one (mean cho_solve, L^-T xi).  Measured
(seeds 901-904, 1500 sweeps): svd chains reach sum(z) ~ 8 within 100-200 sweeps; chol
chains stay at 120-130 for 900-1500+ sweeps -- the reference leaves the trap through its
SVD's error at cond(Sigma) ~ 1e22, not through the model.  See tests/test_gpu_ks.py.
"""
import sys, warnings, numpy as np, scipy.linalg as sl
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from golden_io import load_dataset
from oracle.gibbs_oracle import Oracle, OutlierModel, LegacyNumpyVariates, initial_state
from gibbs_student_t_amd.run_sims import MODELS
warnings.simplefilter("ignore")
mode, seed = sys.argv[1], int(sys.argv[2])
pta = load_dataset(); cfg = OutlierModel(**MODELS["vvh17"])
orc = Oracle(pta, cfg)
if mode == "chol":
    def draw_b(st, x, src, mean="svd"):
        Sigma, d = orc.sigma_matrix(st, x)
        L = np.linalg.cholesky(Sigma)
        mn = sl.cho_solve((L, True), d)
        return mn + sl.solve_triangular(L.T, np.random.randn(len(d)), lower=False)
    orc.draw_b = draw_b
np.random.seed(seed)
x = pta.sample_params(); st = initial_state(pta, cfg); src = LegacyNumpyVariates()
out = []
for i in range(1500):
    x = orc.sweep(st, x, src)
    if i % 100 == 99: out.append(int(np.sum(st.z)))
print(mode, seed, out)
