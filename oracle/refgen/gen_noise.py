"""Noise-parameter fitting fixtures (reference run, container only).

* wls_noise   : a white-noise C5-template pulsar (fixture wls_noise, seed 7) with EFAC1 and
                EQUAD1 free: the white-noise
                lnlikelihood gradient (residuals.py:718-828 d_lnlikelihood_d_param) at the
                par-file values, and DownhillWLSFitter.fit_toas with the noise fit
                (fitter.py:1107-1273: alternating timing / Newton-CG noise fits with the
                analytic gradient).
* ecorr_noise : the ecorr_phoff pulsar with EFAC1 and ECORR1 free: the ECORR-only gradients
                and DownhillGLSFitter.fit_toas (Nelder-Mead noise fit).
* lnl_points  : Residuals.lnlikelihood (residuals.py:713) of fixed residuals at the par values
                and at two perturbed noise points, as _fit_noise evaluates it (fitter.py:1239-1247:
                one Residuals object, its model's noise values changed): wls_noise (diagonal N),
                ecorr_phoff (ECORR Sherman-Morrison), j0740 (ECORR + offset column), pta_iso
                and b1855 (Woodbury with PLRedNoise).
* white_mjd   : tests/test_noisefit.py:10-22's white-noise pulsar (EFAC on mjd 50000-53000,
                EQUAD on mjd 53000-55000, both free; EPHEM builtin for the offline run), 200
                fake TOAs seed 11: DownhillWLSFitter fits from the par values and from
                EFAC 1.5 / EQUAD 0.5 (test_white_noise_fit / test_white_noise_refit).
* ecorr_fit   : tests/datafile/ecorr_fit_test.par/.tim (ECORR and EFAC on tel arecibo,
                PHOFF free): DownhillGLSFitter fits from the par values and from ECORR 0.75
                (test_ecorr_fit / test_ecorr_refit).
compute_noise_uncertainties=False: the reference's Hessian needs numdifftools, which is not
installed here.  Writes tests/golden/noise_fit.json.  Usage: run_ref.sh gen_noise.py
"""
import copy
import io
import json
import os
import sys

import numpy as np
import astropy.units as u

from refcommon import GOLDEN, register_clockless_sites, split_ld
import pint.simulation as sim
from pint.models import get_model
from pint.residuals import Residuals
from pint.fitter import DownhillWLSFitter, DownhillGLSFitter
from gen_phoff import par_phoff
from gen_synth import pta_par, capture


def par_white(seed):
    return "\n".join(l for l in pta_par(seed, "").splitlines() if not l.startswith("TNRed")) + "\n"


def toas_for(seed, ecorr, par=None):
    np.random.seed(seed)
    model = get_model(io.StringIO(par or par_phoff(seed, ecorr)))
    ts = sim.make_fake_toas_uniform(53000, 56652, 600, model,
                                    freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                    obs="geocenter", error=0.5 * u.us, add_noise=True,
                                    add_correlated_noise=ecorr, include_bipm=False,
                                    multi_freqs_in_epoch=ecorr, flags={"f": "fake"})
    model.find_empty_masks(ts, freeze=True)
    return model, ts


def case(name, seed, ecorr, free_noise, fitter_cls, base_name):
    if base_name == "wls_noise":  # its own fixture: white noise only, no PhaseOffset
        par = par_white(seed)
        model, ts = toas_for(seed, False, par)
        with open(os.path.join(GOLDEN, "wls_noise.par"), "w") as f:
            f.write(par)
        capture("wls_noise", copy.deepcopy(model), ts, fit="wls")
    else:
        model, ts = toas_for(seed, ecorr)
    base = np.load(os.path.join(GOLDEN, base_name + ".npz"))
    assert np.array_equal(np.asarray(ts.table["tdbld"], dtype=np.float64), base["tdb_hi"]), "TOAs differ"
    for p in free_noise:
        getattr(model, p).frozen = False
    r = Residuals(ts, copy.deepcopy(model))
    out = {"free_noise": free_noise, "lnlikelihood0": float(r.lnlikelihood()), "grad0": {}, "grad0_error": {}}
    for p in free_noise:
        try:
            out["grad0"][p] = float(r.d_lnlikelihood_d_param(p).value)
        except Exception as e:  # residuals.py:757-781 (EFAC/EQUAD with ECORR) cannot broadcast
            out["grad0_error"][p] = f"{type(e).__name__}: {e}"
    f = fitter_cls(ts, copy.deepcopy(model))
    try:
        f.fit_toas(maxiter=10, compute_noise_uncertainties=False)
        out["status"] = "converged"
    except Exception as e:
        out["status"] = type(e).__name__
    out["chi2"] = float(f.resids.chi2)
    out["lnlikelihood"] = float(f.resids.lnlikelihood())
    out["params"] = {p: list(map(float, split_ld(np.longdouble(getattr(f.model, p).value))))
                     for p in f.model.free_params}
    out["errors"] = {p: (None if getattr(f.model, p).uncertainty_value is None
                         else float(getattr(f.model, p).uncertainty_value)) for p in f.model.free_params}
    print(name, out["status"], out["chi2"], {p: out["params"][p][0] for p in free_noise}, file=sys.stderr)
    return out


WHITE_MJD_PAR = """PSR WHITEMJD
ELAT    1.3     1
ELONG   2.5     1
F0      100     1
F1      1e-13   1
PEPOCH  55000
EPHEM   builtin
EFAC mjd 50000 53000 2      1
EQUAD mjd 53000 55000 0.8    1
"""


def fit_record(f, free_noise):
    out = {}
    try:
        f.fit_toas(maxiter=5 if isinstance(f, DownhillWLSFitter) else 20, compute_noise_uncertainties=False)
        out["status"] = "converged"
    except Exception as e:
        out["status"] = type(e).__name__
    out["chi2"] = float(f.resids.chi2)
    out["lnlikelihood"] = float(f.resids.lnlikelihood())
    out["params"] = {p: list(map(float, split_ld(np.longdouble(getattr(f.model, p).value))))
                     for p in f.model.free_params}
    print(out["status"], out["chi2"], {p: out["params"][p][0] for p in free_noise}, file=sys.stderr)
    return out


def frozen_noise(m):
    """The plain WLS/GLS fitters of capture() cannot take free noise parameters
    (fitter.py:2074): the fixture's free list is the timing parameters; tests free them."""
    m = copy.deepcopy(m)
    for p in m.free_params:
        if p.startswith(("EFAC", "EQUAD", "ECORR")):
            getattr(m, p).frozen = True
    return m


def gen_datafile_cases():
    from refcommon import REFDATA
    import pint.toa as toa
    res = {}
    np.random.seed(11)
    m = get_model(io.StringIO(WHITE_MJD_PAR))
    t = sim.make_fake_toas_uniform(50000, 55000, 200, m, add_noise=True, include_bipm=False)
    with open(os.path.join(GOLDEN, "white_mjd.par"), "w") as f:
        f.write(WHITE_MJD_PAR)
    capture("white_mjd", frozen_noise(m), t, fit="wls")
    free = ["EFAC1", "EQUAD1"]
    res["white_mjd"] = {"free_noise": free, "fit": fit_record(DownhillWLSFitter(t, copy.deepcopy(m)), free)}
    m2 = copy.deepcopy(m)
    m2.EFAC1.value, m2.EQUAD1.value = 1.5, 0.5
    res["white_mjd"]["refit"] = fit_record(DownhillWLSFitter(t, m2), free)
    m = get_model(f"{REFDATA}/ecorr_fit_test.par")
    t = toa.get_TOAs(f"{REFDATA}/ecorr_fit_test.tim", ephem="builtin", include_bipm=False, planets=False, model=m)
    with open(f"{REFDATA}/ecorr_fit_test.par") as fi, open(os.path.join(GOLDEN, "ecorr_fit.par"), "w") as fo:
        fo.write(fi.read())
    capture("ecorr_fit", frozen_noise(m), t, fit="gls")
    free = ["ECORR1", "EFAC1"]
    res["ecorr_fit"] = {"free_noise": free, "truth": {"ECORR1": float(m.ECORR1.value), "EFAC1": float(m.EFAC1.value)},
                        "fit": fit_record(DownhillGLSFitter(t, copy.deepcopy(m)), free)}
    m2 = copy.deepcopy(m)
    m2.ECORR1.value = 0.75
    res["ecorr_fit"]["refit"] = fit_record(DownhillGLSFitter(t, m2), free)
    return res


def perturbations(model):
    """Two trial points: every EFAC x1.1 / x0.9, EQUAD x1.5 / x0.5, ECORR x1.3 / x0.7,
    TNREDAMP +-0.2, TNREDGAM -+0.3."""
    pts = []
    for sgn in (1, -1):
        d = {}
        for n in model.params:
            par = getattr(model, n)
            if par.value is None:
                continue
            if n.startswith("EFAC"):
                d[n] = float(par.value) * (1.1 if sgn > 0 else 0.9)
            elif n.startswith("EQUAD"):
                d[n] = float(par.value) * (1.5 if sgn > 0 else 0.5)
            elif n.startswith("ECORR"):
                d[n] = float(par.value) * (1.3 if sgn > 0 else 0.7)
            elif n == "TNREDAMP":
                d[n] = float(par.value) + 0.2 * sgn
            elif n == "TNREDGAM":
                d[n] = float(par.value) - 0.3 * sgn
        pts.append(d)
    return pts


def lnl_points(model, ts):
    r = Residuals(ts, copy.deepcopy(model))
    out = [{"values": {}, "lnl": float(r.lnlikelihood())}]
    for d in perturbations(model):
        for n, v in d.items():
            getattr(r.model, n).value = v
        out.append({"values": d, "lnl": float(r.lnlikelihood())})
    return out


def all_lnl_points():
    from gen_synth import j0740_model
    from refcommon import REFDATA
    import pint.toa as toa
    res = {}
    np.random.seed(7)
    par = par_white(7)
    res["wls_noise"] = lnl_points(*toas_for(7, False, par))
    res["ecorr_phoff"] = lnl_points(*toas_for(6, True))
    # j0740 / pta_iso exactly as gen_synth.gen_j0740 / gen_pta build them
    np.random.seed(0)
    model = j0740_model()
    ts = sim.make_fake_toas_uniform(56640, 58461, 1000, model, freq=np.array([820, 1400]) * u.MHz,
                                    obs="geocenter", error=1 * u.us, add_noise=False,
                                    include_bipm=False, multi_freqs_in_epoch=False,
                                    flags={"f": "Rcvr1_2_GUPPI", "fe": "Rcvr1_2"})
    for fl, fr in zip(ts.table["flags"], ts.table["freq"]):
        if fr < 1000:
            fl["f"] = "Rcvr_800_GUPPI"
            fl["fe"] = "Rcvr_800"
    ts = sim.make_fake_toas(ts, model, add_noise=True)
    model.find_empty_masks(ts, freeze=True)
    base = np.load(os.path.join(GOLDEN, "j0740.npz"))
    assert np.array_equal(np.asarray(ts.table["tdbld"], dtype=np.float64), base["tdb_hi"]), "j0740 TOAs differ"
    res["j0740"] = lnl_points(model, ts)
    np.random.seed(1)
    model = get_model(io.StringIO(pta_par(1, "")))
    ts = sim.make_fake_toas_uniform(53000, 56652, 1000, model,
                                    freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                    obs="geocenter", error=0.5 * u.us, add_noise=True,
                                    add_correlated_noise=True, include_bipm=False,
                                    multi_freqs_in_epoch=False)
    model.find_empty_masks(ts, freeze=True)
    base = np.load(os.path.join(GOLDEN, "pta_iso.npz"))
    assert np.array_equal(np.asarray(ts.table["tdbld"], dtype=np.float64), base["tdb_hi"]), "pta_iso TOAs differ"
    res["pta_iso"] = lnl_points(model, ts)
    model = get_model(f"{REFDATA}/B1855+09_NANOGrav_9yv1.gls.par")
    ts = toa.get_TOAs(f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", ephem="builtin",
                      include_bipm=False, planets=False, model=model)
    res["b1855"] = lnl_points(model, ts)
    for k, v in res.items():
        print(k, [p["lnl"] for p in v], file=sys.stderr)
    return res


if __name__ == "__main__":
    register_clockless_sites()
    res = {"wls_noise": case("wls_noise", 7, False, ["EFAC1", "EQUAD1"], DownhillWLSFitter, "wls_noise"),
           "ecorr_noise": case("ecorr_noise", 6, True, ["EFAC1", "ECORR1"], DownhillGLSFitter, "ecorr_phoff"),
           "lnl_points": all_lnl_points()}
    res.update(gen_datafile_cases())
    with open(os.path.join(GOLDEN, "noise_fit.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
