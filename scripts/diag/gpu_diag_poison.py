"""Diagnostic (not a test): which outputs turn NaN for a GLS step under PINT_CACHE_POISON=1."""
import copy, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from golden_util import load
from pint_amd.fitter import BatchFit
for name in sys.argv[1:]:
    model, toas, z, meta = load(name)
    for blocked in (True, False):
        bf = BatchFit([(copy.deepcopy(model), toas)], mode="gls")
        bf.s.set_blocked_solve(blocked)
        lay = bf.layouts[0]
        print(name, "blocked", blocked, "n", lay.n, "K", lay.K, "nred", lay.nred, "nep", lay.nep, flush=True)
        bf.s.eval(want_M=bf.s.FIT)
        tr, pr, c2 = bf.s.read_resids()
        print("  eval: nan tr", np.isnan(tr[0]).sum(), "chi2", c2, flush=True)
        bf.s.fit_step(1)
        dp, er, cov, cl = bf.s.read_step()
        print("  step: nan dp", np.isnan(dp[0]).sum(), "er", np.isnan(er[0]).sum(), "cov", np.isnan(cov[0]).sum(),
              "chi2lin", cl, flush=True)
        print("  chi2_gls", bf.s.chi2_gls(), "lognorm", bf.s.lognorm(1), flush=True)
        bf.close()
