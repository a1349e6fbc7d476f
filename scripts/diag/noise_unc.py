import sys
sys.path[:0] = [".", "tests", "oracle"]
import numpy as np
from golden_util import load
import pint_amd.fitter as F
from pint_amd.noisefit import NoiseLikelihood, hessian, fit_noise
model, toas, z, meta = load("wls_noise")
for p in ("EFAC1", "EQUAD1"):
    model[p].frozen = False
f = F.DownhillWLSFitter(toas, model)
f.fit_toas(maxiter=10, compute_noise_uncertainties=True)
print("vals", [f.model[p].value for p in ("EFAC1", "EQUAD1")], "errs", [f.model[p].uncertainty_value for p in ("EFAC1", "EQUAD1")])
nl = NoiseLikelihood(toas, f.model, ["EFAC1", "EQUAD1"])
x = np.array([float(f.model[p].value) for p in nl.params])
print("lnl", nl.lnlikelihood(x), "grad", nl.d_lnlikelihood_d_params(x))
H = hessian(lambda xs: -nl.lnlikelihood(xs), x)
print("H", H, np.linalg.eigvalsh(H))
for d in (-1e-3, 1e-3):
    print(d, nl.lnlikelihood(x + [d, 0]), nl.lnlikelihood(x + [0, d]))
v, e = fit_noise(toas, f.model, uncertainty=True)
print("refit", v, e)
