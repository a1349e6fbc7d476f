"""Noise-parameter fitting: DownhillFitter._fit_noise's likelihood of
fixed residuals (fitter.py:1230-1273, residuals.py:591-828) and the fits themselves, against
tests/golden/noise_fit.json (oracle/refgen/gen_noise.py, the reference run in the build
container).

CPU tests pin the oracle's restatement; GPU tests run the product (k_noise_lnl through
pint_noise_lnlike, the Woodbury path through pint_set_sigma / pint_set_noise_weights) and
compare with the reference and the oracle."""
import copy
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN, load
import pint_oracle as O
from test_oracle_golden import fixture

NOISE = json.load(open(os.path.join(GOLDEN, "noise_fit.json")))
POINT_NAMES = ["wls_noise", "ecorr_phoff", "j0740", "pta_iso", "b1855"]


def _with(om, values):
    om2 = copy.deepcopy(om)
    for k, v in values.items():
        om2.values[k] = v
    return om2


@pytest.mark.parametrize("name", POINT_NAMES)
def test_oracle_lnl_points(name):
    """The oracle's likelihood of the reference's own residuals at the reference's trial
    noise points (diagonal, Sherman-Morrison, offset-column and Woodbury branches)."""
    om, toas, z, meta = fixture(name)
    for pt in NOISE["lnl_points"][name]:
        ll = O.lnlikelihood_of(_with(om, pt["values"]), toas, z["res_time"])
        assert abs(ll - pt["lnl"]) < 1e-9 * abs(pt["lnl"]), (pt["values"], ll, pt["lnl"])


def test_oracle_white_gradient():
    """residuals.py:809-828 for EFAC/EQUAD at the par values (reference d_lnlikelihood_d_param)."""
    om, toas, z, meta = fixture("wls_noise")
    ref = NOISE["wls_noise"]
    assert abs(O.lnlikelihood_of(om, toas, z["res_time"]) - ref["lnlikelihood0"]) < 1e-9 * abs(ref["lnlikelihood0"])
    for p, g in ref["grad0"].items():
        mine = O.d_lnlikelihood_d_param(om, toas, z["res_time"], p)
        assert abs(mine - g) < 1e-9 * abs(g), (p, mine, g)


def test_reference_ecorr_gradients_broken():
    """The reference's ECORR-branch gradients do not run in this version (recorded by the
    generator): the product computes the correct derivatives, pinned by finite differences."""
    err = NOISE["ecorr_noise"]["grad0_error"]
    assert set(err) == {"EFAC1", "ECORR1"}
    assert "broadcast" in err["EFAC1"] and "UnitConversionError" in err["ECORR1"]


# ---------------------------------------------------------------------------------------
# GPU: the product
# ---------------------------------------------------------------------------------------
def _nl(name, params, ref_resids=True):
    from pint_amd.noisefit import NoiseLikelihood
    model, toas, z, meta = load(name)
    for p in params:
        model[p].frozen = False
    nl = NoiseLikelihood(toas, model, params)
    if ref_resids:
        nl.set_resids(z["res_time"])
    return nl, model, toas, z, meta


def _point_params(name):
    pts = NOISE["lnl_points"][name]
    return sorted(pts[1]["values"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", POINT_NAMES)
def test_lnl_points(name):
    """Stage-wise (the reference's residuals on the device): lnL at the reference's trial
    points to 1e-10 relative; end-to-end (the device's own residuals): within the residual
    floor (~1e-6 of chi2)."""
    from pint_amd.noisefit import likelihood_kind
    params = _point_params(name)
    nl, model, toas, z, meta = _nl(name, params)
    try:
        assert nl.kind == {"wls_noise": 0, "ecorr_phoff": 1, "j0740": 2, "pta_iso": 3, "b1855": 3}[name]
        for pt in NOISE["lnl_points"][name]:
            xs = [pt["values"].get(p, float(model[p].value)) for p in params]
            ll = nl.lnlikelihood(xs)
            assert abs(ll - pt["lnl"]) < 1e-10 * abs(pt["lnl"]), (pt["values"], ll, pt["lnl"], ll - pt["lnl"])
    finally:
        nl.close()
    nl2, model, toas, z, meta = _nl(name, params, ref_resids=False)
    try:
        ll = nl2.lnlikelihood()
        ref = NOISE["lnl_points"][name][0]["lnl"]
        assert abs(ll - ref) < 1e-6 * abs(meta["res_chi2"]) + 1e-9 * abs(ref), (ll, ref)
    finally:
        nl2.close()


@pytest.mark.gpu
def test_white_gradient():
    """d_lnlikelihood_d_param for EFAC1/EQUAD1 (residuals.py:809-828) against the reference,
    and against central differences of the device likelihood."""
    nl, model, toas, z, meta = _nl("wls_noise", ["EFAC1", "EQUAD1"])
    try:
        ref = NOISE["wls_noise"]
        x0 = [float(model["EFAC1"].value), float(model["EQUAD1"].value)]
        assert abs(nl.lnlikelihood(x0) - ref["lnlikelihood0"]) < 1e-10 * abs(ref["lnlikelihood0"])
        g = nl.d_lnlikelihood_d_params(x0)
        for k, p in enumerate(nl.params):
            assert abs(g[k] - ref["grad0"][p]) < 1e-9 * abs(ref["grad0"][p]), (p, g[k], ref["grad0"][p])
        _check_fd(nl, x0, g)
    finally:
        nl.close()


def _check_fd(nl, x0, g, rel=1e-6):
    for k in range(len(x0)):
        h = 1e-4 * max(abs(x0[k]), 0.1)
        xp, xm = list(x0), list(x0)
        xp[k] += h
        xm[k] -= h
        fd = (nl.lnlikelihood(xp) - nl.lnlikelihood(xm)) / (2 * h)
        assert abs(fd - g[k]) < rel * max(abs(g[k]), 1.0) + 1e-6, (nl.params[k], fd, g[k])


@pytest.mark.gpu
def test_ecorr_gradient_fd():
    """The ECORR-only (Sherman-Morrison) gradients: EFAC1 and ECORR1 against central
    differences of the reference-pinned likelihood (the reference's own branches fail,
    test_reference_ecorr_gradients_broken)."""
    nl, model, toas, z, meta = _nl("ecorr_phoff", ["EFAC1", "ECORR1"])
    try:
        for scale in (1.0, 1.3):
            x0 = [float(model["EFAC1"].value), float(model["ECORR1"].value) * scale]
            _check_fd(nl, x0, nl.d_lnlikelihood_d_params(x0))
    finally:
        nl.close()


@pytest.mark.gpu
def test_gradient_not_implemented():
    """residuals.py:812-816: no gradient with time-correlated noise or without a free PHOFF."""
    for name in ("pta_iso", "j0740"):
        params = _point_params(name)
        nl, *_ = _nl(name, params)
        try:
            with pytest.raises(NotImplementedError):
                nl.d_lnlikelihood_d_params()
        finally:
            nl.close()


@pytest.mark.gpu
def test_batch_lnlike():
    """One k_noise_lnl launch over two pulsars of different kinds: per-instance class and
    epoch offsets."""
    from pint_amd.engine import Session, build_layout, pack_table
    from pint_amd.noisefit import white_noise_classes
    outs = []
    for name in ("wls_noise", "ecorr_phoff"):
        nl, *_ = _nl(name, _point_params(name))
        outs.append((nl.lnlikelihood(), nl.d_lnlikelihood_d_params(), nl))
    s = Session()
    try:
        lays, qfs, eps = [], [], []
        for name in ("wls_noise", "ecorr_phoff"):
            model, toas, z, meta = load(name)
            for p in _point_params(name):
                model[p].frozen = False
            lay = s.add(build_layout(model, toas))
            ptr, idx, _, _ = white_noise_classes(model, toas)
            s.set_noise_classes(lay, ptr, idx, toas.get_errors())
            lays.append((lay, z))
        s.set_instances([(lay, pack_table(lay)) for lay, _ in lays])
        s.set_resids([z["res_time"] for _, z in lays])
        for _, _, nl in outs:
            qfs.append(nl._qf())
            w = nl._ep_w()
            if w is not None:
                eps.append(w)
        out, g, eg = s.noise_lnlike([0, 1], np.vstack(qfs), np.concatenate(eps))
        for k, (ll, _, _) in enumerate(outs):
            assert abs(out[k, 0] - ll) < 1e-12 * abs(ll)
    finally:
        s.close()
        for *_, nl in outs:
            nl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case,fitter", [("wls_noise", "DownhillWLSFitter"), ("ecorr_noise", "DownhillGLSFitter")])
def test_noise_fit(case, fitter):
    """DownhillFitter.fit_toas with free noise parameters (fitter.py:1107-1204): alternating
    timing fits and device noise fits (Newton-CG with the analytic gradient for white noise,
    Nelder-Mead with ECORR), against the reference run."""
    import pint_amd.fitter as F
    ref = NOISE[case]
    name = {"wls_noise": "wls_noise", "ecorr_noise": "ecorr_phoff"}[case]
    model, toas, z, meta = load(name)
    for p in ref["free_noise"]:
        model[p].frozen = False
    f = getattr(F, fitter)(toas, model)
    f.fit_toas(maxiter=10, compute_noise_uncertainties=False)
    assert ref["status"] == "converged"
    # Newton-CG stops at xtol 1e-5 relative, Nelder-Mead at xatol 1e-4: the two optima
    # agree to those tolerances
    tol = 3e-5 if case == "wls_noise" else 3e-4
    for p in ref["free_noise"]:
        v, rv = float(f.model[p].value), ref["params"][p][0]
        assert abs(v - rv) < tol * abs(rv), (p, v, rv)
    assert abs(f.resids.chi2 - ref["chi2"]) < 1e-4 * ref["chi2"], (f.resids.chi2, ref["chi2"])
    assert abs(f.resids.lnlikelihood() - ref["lnlikelihood"]) < 1e-3, (f.resids.lnlikelihood(), ref["lnlikelihood"])
    for p, (hi, lo) in ref["params"].items():
        if p in ref["free_noise"]:
            continue
        sig = float(f.model[p].uncertainty_value)
        assert abs(float(np.longdouble(f.model[p].value) - (np.longdouble(hi) + np.longdouble(lo)))) < 0.05 * sig, p


@pytest.mark.gpu
def test_noise_uncertainties():
    """compute_noise_uncertainties: errors = sqrt(diag(pinv(H))), H the Hessian of -lnL
    (fitter.py:1269-1271).  numdifftools is absent here, so H is noisefit.hessian's
    Richardson-extrapolated central difference; pinned by the closed form of a one-EFAC
    likelihood, H = 3 sum r^2 / (N0 F^4) - n / F^2 (N0 = sigma0^2 + EQUAD^2)."""
    import pint_amd.fitter as F
    from pint_amd.noisefit import NoiseLikelihood
    model, toas, z, meta = load("wls_noise")
    model["EFAC1"].frozen = False
    f = F.DownhillWLSFitter(toas, model)
    f.fit_toas(maxiter=10, compute_noise_uncertainties=True)
    err = f.model["EFAC1"].uncertainty_value
    # closed form at the fitted EFAC with the final residuals (the error was taken before the
    # last timing fit, which moves the residuals by << their uncertainty)
    nl = NoiseLikelihood(toas, f.model, ["EFAC1"])
    try:
        r = nl.time_resids
    finally:
        nl.close()
    Fv = float(f.model["EFAC1"].value)
    N0 = ((toas.get_errors() ** 2 + float(f.model["EQUAD1"].value) ** 2) * 1e-12)
    H = 3 * np.sum(r ** 2 / N0) / Fv ** 4 - len(r) / Fv ** 2
    assert abs(err * np.sqrt(H) - 1) < 1e-3, (err, 1 / np.sqrt(H))
    # at the optimum of a single EFAC: F^2 = sum(r^2/N0)/n, so H = 2n/F^2
    assert abs(Fv ** 2 / (np.sum(r ** 2 / N0) / len(r)) - 1) < 1e-4


@pytest.mark.gpu
def test_noise_uncertainties_degenerate():
    """EFAC1 and EQUAD1 of equal-error TOAs are degenerate (only F^2 (sigma0^2 + Q^2)
    matters): the Hessian has a zero eigenvalue up to rounding, so sqrt(diag(pinv(H)))
    (fitter.py:1270-1271) is huge where the rounding leaves it positive and NaN where it
    leaves it negative -- which of the two depends on the last bits of the residual sums (a
    change of the residual pass's summation order flipped it), in the reference as here.
    Never a small, confident error."""
    import pint_amd.fitter as F
    model, toas, z, meta = load("wls_noise")
    for p in ("EFAC1", "EQUAD1"):
        model[p].frozen = False
    f = F.DownhillWLSFitter(toas, model)
    f.fit_toas(maxiter=10, compute_noise_uncertainties=True)
    errs = [f.model[p].uncertainty_value for p in ("EFAC1", "EQUAD1")]
    assert all(e is not None and (np.isnan(e) or e > 1.0) for e in errs), errs


# ---------------------------------------------------------------------------------------
# the reference's own noise-fit tests (tests/test_noisefit.py) on their inputs
# ---------------------------------------------------------------------------------------
def _fit_case(name, fitter, start=None, maxiter=None):
    import pint_amd.fitter as F
    model, toas, z, meta = load(name)
    ref = NOISE[name]
    for p in ref["free_noise"]:
        model[p].frozen = False
    for p, v in (start or {}).items():
        model[p].value = v
    f = getattr(F, fitter)(toas, model)
    f.fit_toas(**({"maxiter": maxiter} if maxiter else {}))
    return f, ref


def _check_against(f, rec, free, tol):
    assert rec["status"] == "converged"
    for p in free:
        v, rv = float(f.model[p].value), rec["params"][p][0]
        assert abs(v - rv) < tol * abs(rv), (p, v, rv)
    assert abs(f.resids.chi2 - rec["chi2"]) < 1e-4 * rec["chi2"], (f.resids.chi2, rec["chi2"])


@pytest.mark.gpu
@pytest.mark.parametrize("start", [None, {"EFAC1": 1.5, "EQUAD1": 0.5}])
def test_white_noise_fit_mjd_masks(start):
    """test_noisefit.py:29-67 (test_white_noise_fit / _refit): EFAC on an MJD range and EQUAD
    on another, fitted with uncertainties; within 4 sigma of the simulated values and equal
    to the reference's fit (its run without uncertainties: numdifftools is absent)."""
    f, ref = _fit_case("white_mjd", "DownhillWLSFitter", start, maxiter=5)
    for p, truth in (("EFAC1", 2.0), ("EQUAD1", 0.8)):
        err = f.model[p].uncertainty_value
        assert err is not None and err > 0
        assert abs(float(f.model[p].value) - truth) / err < 4, (p, f.model[p].value, err)
    _check_against(f, ref["refit" if start else "fit"], ref["free_noise"], 3e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("start", [None, {"ECORR1": 0.75}])
def test_ecorr_fit_tel_masks(start):
    """test_noisefit.py:70-94 (test_ecorr_fit / _refit) on ecorr_fit_test.par/.tim: ECORR and
    EFAC on 'tel arecibo' with PHOFF free, Nelder-Mead on the Sherman-Morrison likelihood.
    The fixture's TOAs were prepared with the builtin ephemeris (offline), so the epoch-
    correlated ephemeris error moves ECORR far from the value the data file was simulated
    with; the check is against the reference's own fit of the same TOAs."""
    f, ref = _fit_case("ecorr_fit", "DownhillGLSFitter", start)
    assert f.model["ECORR1"].uncertainty_value > 0
    _check_against(f, ref["refit" if start else "fit"], ref["free_noise"], 3e-4)
