import sys, copy, numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from golden_util import load
from pint_amd import GLSFitter, Residuals
from pint_amd.engine import Session
from pint_amd.fitter import BatchFit
model, toas, z, meta = load("pta_dd")
e0 = float(model.ECC.value)
for fac in (1.0, 1 + 1e-7, 1 + 1e-5, 1.001):
    m = copy.deepcopy(model); m.ECC.value = e0 * fac; m.ECC.frozen = True
    r = Residuals(toas, m)
    print(fac, "resid rms", np.std(r.time_resids), "chi2", r.chi2)
    bf = BatchFit([(m, toas)], mode="gls")
    bf.s.eval(want_M=Session.FIT)
    bf.s.fit_step(1)
    dp, er, cov, cl = bf.s.read_step()
    print("  dp finite", np.all(np.isfinite(dp[0])), "err finite", np.all(np.isfinite(er[0])), "chi2lin", cl)
    print("  chi2_gls pre", bf.s.chi2_gls())
    bf.s.apply_step(np.ones(1)); bf.s.eval(False)
    tr, pr, c2 = bf.s.read_resids()
    print("  post wls chi2", c2, "gls", bf.s.chi2_gls(), "resid finite", np.all(np.isfinite(tr[0])))
    bf.close()
