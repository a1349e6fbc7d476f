import sys, numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from golden_util import load
from pint_amd.noise import fourier_basis
from pint_amd.engine import Session
from pint_amd.fitter import BatchFit
model, toas, z, meta = load("b1855")
st = dict(np.load("tests/golden/b1855_stage.npz"))
F = fourier_basis(model, toas).astype(np.float64)
bf = BatchFit([(model, toas)], mode="gls")
s = bf.s
s.eval(want_M=True)
M = s.read_designmatrix()[0]
lay = bf.layouts[0]
nc = len(lay.columns)
Fd = M[:, nc:]
print("F max abs diff", np.max(np.abs(Fd - F)), "cols", Fd.shape)
s.eval(want_M=Session.FIT)
s.debug_set_resids([z["res_time"]])
s.fit_step(1)
G, colsq = s.debug_gram()[0]
Gp, _ = s.debug_gram(pre_ecorr=True)[0]
nh = np.sqrt(np.sum(F ** 2, axis=0))
print("colsq vs host F norms", np.max(np.abs(np.sqrt(colsq[nc:]) / nh - 1)))
tr = st["cols_tr"]
print("colsq vs ref norms (timing)", np.max(np.abs(np.sqrt(colsq[:nc]) / st["norm"][tr][:nc] - 1)))
print("colsq vs ref norms (red)", np.max(np.abs(np.sqrt(colsq[nc:]) / st["norm"][tr][nc:] - 1)))
w = 1 / (lay.sigma_us * 1e-6) ** 2
Gh = (F * w[:, None]).T @ F
K = lay.K
print("Gram red block (pre-ECORR) vs host float64:", np.max(np.abs(Gp[nc:K, nc:K] - Gh) / np.sqrt(np.outer(np.diag(Gh), np.diag(Gh)))))
