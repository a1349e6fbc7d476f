"""(diagnostic) The measured distance of the GPU DownhillGLSFitter parameters from the
reference's (in reference sigmas), and of the GLS uncertainties, per fixture: the margins
behind the bars of tests/test_gpu_parity.py."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from golden_util import load, ref_value  # noqa: E402
from pint_amd import DownhillGLSFitter, GLSFitter  # noqa: E402
from pint_amd.fitter import MaxiterReached, StepProblem  # noqa: E402

for name in ["pta_iso", "pta_ell1", "pta_dd", "ecorr_phoff", "j0740"]:
    model, toas, z, meta = load(name)
    if "down_params" not in meta:
        continue
    f = DownhillGLSFitter(toas, model)
    try:
        f.fit_toas(maxiter=10)
    except (MaxiterReached, StepProblem):
        pass
    ds = {p: float((np.longdouble(f.model[p].value) - ref_value(meta, "down_params", p)) / np.longdouble(meta["down_errors"][p]))
          for p in meta["down_params"]}
    w = max(ds, key=lambda p: abs(ds[p]))
    es = {p: abs(f.model[p].uncertainty / meta["down_errors"][p] - 1) for p in meta["down_params"]}
    we = max(es, key=es.get)
    print(f"downhill {name}: worst param {w} {ds[w]:.3e} sigma; worst error {we} {es[we]:.3e}; "
          f"chi2 {f.resids.chi2 / meta['down_chi2'] - 1:.2e}", flush=True)
for name in ["j0740", "b1855"]:
    model, toas, z, meta = load(name)
    f = GLSFitter(toas, model)
    f.fit_toas(maxiter=1)
    es = {p: abs(f.model[p].uncertainty / meta["gls_errors"][p] - 1) for p in meta["gls_params"]}
    we = max(es, key=es.get)
    print(f"gls {name}: worst uncertainty {we} {es[we]:.3e}", flush=True)
