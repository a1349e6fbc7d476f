"""The reference's own Downhill spread under ps-level residual perturbations (reference run;
container only; TEST INFRASTRUCTURE).

Two longdouble / double-double evaluations of the same model differ by about 5 ps rms per
TOA (SURVEY.md finding 3).  DownhillGLSFitter picks its best iterate by
comparing chi2 values, so a parameter along a nearly degenerate direction (pta_dd's M2 /
SINI Shapiro pair) can move by more than 1e-3 sigma under such a perturbation.  This script
measures that for the reference itself: it reruns DownhillGLSFitter.fit_toas(maxiter=10) on
the fixture with every time residual the reference computes (Residuals.calc_time_resids,
residuals.py:483) shifted by a fixed per-TOA N(0, 5 ps) draw (seeds 1..NREP) -- a shift of
the TOAs themselves is below tdbld's longdouble resolution (0.5 ns at MJD 5e4) -- and
records, per fitted parameter, max |p_perturbed - p_unperturbed| / sigma.
tests/test_gpu_parity.py::test_downhill_gls sets its per-parameter bar from it.

wb_dd runs WidebandDownhillFitter (fitter.py:1812-1895) the same way; its TOA residuals
(WidebandTOAResiduals.toa) are the perturbed ones.

Usage: oracle/refenv/run_ref.sh oracle/refgen/gen_downhill_spread.py [name ...]
Writes tests/golden/downhill_spread.json.
"""
import copy
import json
import os
import sys

import numpy as np

from refcommon import GOLDEN, register_clockless_sites
import astropy.units as u
import pint.fitter as pfit
import pint.residuals as pres

from gen_stage import rebuild

NREP = 8
SIGMA_S = 5e-12


def fit(model, toas, cls=pfit.DownhillGLSFitter):
    f = cls(toas, copy.deepcopy(model))
    try:
        f.fit_toas(maxiter=10)
        status = "converged"
    except Exception as e:
        status = type(e).__name__
    vals = {p: np.longdouble(getattr(f.model, p).value) for p in f.model.free_params}
    errs = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
    return vals, errs, status, float(f.resids.chi2)


def spread(name):
    cls = pfit.DownhillGLSFitter
    if name == "wb_dd":  # WidebandDownhillFitter; the TOA part of its residuals is perturbed
        import gen_wideband
        _, model, toas = gen_wideband.build()
        cls = pfit.WidebandDownhillFitter
    else:
        model, toas = rebuild(name)
    v0, e0, s0, c0 = fit(model, toas, cls)
    worst = {p: 0.0 for p in v0}
    statuses, chi2s = [], []
    orig = pres.Residuals.calc_time_resids
    try:
        for rep in range(1, NREP + 1):
            delta = np.random.default_rng(rep).normal(size=len(toas)) * SIGMA_S

            def calc(self, *a, **k):
                return orig(self, *a, **k) + delta * u.s

            pres.Residuals.calc_time_resids = calc
            v, e, s, c = fit(model, toas, cls)
            statuses.append(s)
            chi2s.append(c / c0 - 1)
            for p in v0:
                worst[p] = max(worst[p], abs(float((v[p] - v0[p]) / np.longdouble(e0[p]))))
    finally:
        pres.Residuals.calc_time_resids = orig
    return {"sigma_s": SIGMA_S, "nrep": NREP, "status": s0, "statuses": statuses,
            "chi2_rel": [float(x) for x in chi2s], "max_dev_sigma": worst}


if __name__ == "__main__":
    register_clockless_sites()
    out = {}
    path = os.path.join(GOLDEN, "downhill_spread.json")
    if os.path.exists(path):
        out = json.load(open(path))
    for n in sys.argv[1:] or ["pta_dd"]:
        out[n] = spread(n)
        w = out[n]["max_dev_sigma"]
        top = sorted(w.items(), key=lambda kv: -kv[1])[:5]
        print(n, top, file=sys.stderr)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
