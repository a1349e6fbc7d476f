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
    with open(os.path.join(GOLDEN, "noise_fit.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
