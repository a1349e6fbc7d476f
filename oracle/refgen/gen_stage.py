"""Stage-wise golden fixtures (reference run; container only; TEST INFRASTRUCTURE).

For every GLS fixture this captures the arrays GLSFitter.fit_toas forms inside its first
iteration (/root/reference/src/pint/fitter.py:2164-2202), exactly as the reference's own
code computes them:

* mtcm   the normalised normal matrix M^T N^-1 M + diag(phiinv / norm^2)  (:2187-2192)
* mtcy   M^T N^-1 r                                                        (:2193)
* xhat   cho_solve(mtcm, mtcy), xvar = cho_solve(mtcm, I)                 (:2196-2202)
* norm   normalize_designmatrix's column norms                             (:2176-2177)
* phiinv the normalised prior inverse on the noise columns                (:2185)
* noise_resids of the fit                                                  (:2270-2282)

mtcm/mtcy/xhat/xvar are recorded by wrapping scipy.linalg.cho_factor / cho_solve for the
duration of that one call, so the values are the reference's arrays, not a restatement.
The residuals r of that iteration are the pre-fit `Residuals(toas, model).time_resids`,
which the base fixture already holds as `res_time`.

For j0740 it also runs the C4 (M2, SINI) grid: 5 x 5, M2 in [0.2, 0.3] Msun, SINI =
sin(86.25..88.5 deg) (profiling/bench_chisq_grid.py:33-35 ranges), GLSFitter per point,
both serial (ncpu=1, warm start) and parallel (ncpu=2, cold start) (gridutils.py:166-389).

The models and TOAs are rebuilt by the same recipes as gen_synth.py / gen_b1855.py, and the
packed tdb of the rebuilt TOAs is checked bit-for-bit against the committed base fixture.

Usage: oracle/refenv/run_ref.sh oracle/refgen/gen_stage.py [name ...]
Writes tests/golden/<name>_stage.npz.
"""
import copy
import os
import sys

import numpy as np
import astropy.units as u
import scipy.linalg

from refcommon import GOLDEN, REFDATA, register_clockless_sites, pack_toas, split_ld
import pint.fitter as pfit
import pint.simulation as sim
import pint.toa as toa
from pint.models import get_model
from pint.gridutils import grid_chisq

import gen_synth


def rebuild(name):
    """(model, toas) of a base fixture, by its generator's recipe."""
    if name == "b1855":
        model = get_model(f"{REFDATA}/B1855+09_NANOGrav_9yv1.gls.par")
        toas = toa.get_TOAs(f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", ephem="builtin",
                            include_bipm=False, planets=False, model=model)
        return model, toas
    if name == "j0740":
        np.random.seed(0)
        model = gen_synth.j0740_model()
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
        return model, ts
    seed, binary = {"pta_iso": (1, ""), "pta_ell1": (2, "ELL1"), "pta_dd": (3, "DD")}[name]
    np.random.seed(seed)
    import io
    model = get_model(io.StringIO(gen_synth.pta_par(seed, binary)))
    ts = sim.make_fake_toas_uniform(53000, 56652, 1000, model, freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                    obs="geocenter", error=0.5 * u.us, add_noise=True,
                                    add_correlated_noise=True, include_bipm=False, multi_freqs_in_epoch=False)
    model.find_empty_masks(ts, freeze=True)
    return model, ts


def check_same_toas(name, toas):
    base = np.load(os.path.join(GOLDEN, name + ".npz"))
    arr, _ = pack_toas(toas)
    for k in ("tdb_hi", "tdb_lo", "freq_mhz", "err_us"):
        if not np.array_equal(arr[k], base[k]):
            raise SystemExit(f"{name}: rebuilt TOAs differ from the committed fixture in {k}")


class Recorder:
    """Wraps scipy.linalg.cho_factor / cho_solve (the calls of fitter.py:2196-2199)."""

    def __init__(self):
        self.calls = []

    def __enter__(self):
        self._cf, self._cs = scipy.linalg.cho_factor, scipy.linalg.cho_solve
        rec = self

        def cf(a, *args, **kw):
            rec.calls.append(("cho_factor", np.array(a, dtype=np.float64)))
            return rec._cf(a, *args, **kw)

        def cs(c, b, *args, **kw):
            x = rec._cs(c, b, *args, **kw)
            rec.calls.append(("cho_solve", np.array(b, dtype=np.float64), np.array(x, dtype=np.float64)))
            return x

        scipy.linalg.cho_factor, scipy.linalg.cho_solve = cf, cs
        return self

    def __exit__(self, *a):
        scipy.linalg.cho_factor, scipy.linalg.cho_solve = self._cf, self._cs


def stage(name):
    model, toas = rebuild(name)
    check_same_toas(name, toas)
    out = {}
    f = pfit.GLSFitter(toas, copy.deepcopy(model))
    with Recorder() as rec:
        chi2 = f.fit_toas(maxiter=1, debug=True)
    kinds = [c[0] for c in rec.calls]
    assert kinds[:3] == ["cho_factor", "cho_solve", "cho_solve"], kinds
    mtcm = rec.calls[0][1]
    mtcy, xhat = rec.calls[1][1], rec.calls[1][2]
    xvar = rec.calls[2][2]
    norm = np.asarray(f.resids.norm, dtype=np.float64)
    K = mtcm.shape[0]
    out["K"] = np.array([K])
    out["mtcy"] = mtcy
    out["xhat"] = xhat
    dims = model.noise_model_dimensions(toas)
    ntm = len(f.model.free_params) + 1
    # columns kept by the device path: timing + red noise; the ECORR quantisation block
    # is eliminated there (its normal-matrix block is diagonal: disjoint epochs)
    ecorr = np.zeros(K, dtype=bool)
    for c, (a, b) in dims.items():
        if c == "ecorr_noise":
            ecorr[ntm + a:ntm + a + b] = True
    tr = np.where(~ecorr)[0]
    ec = np.where(ecorr)[0]
    out["cols_tr"] = tr
    out["cols_ecorr"] = ec
    Mtt = mtcm[np.ix_(tr, tr)]
    out["mtcm_tr_triu"] = Mtt[np.triu_indices(len(tr))]
    if len(ec):
        Mee = mtcm[np.ix_(ec, ec)]
        assert np.count_nonzero(Mee - np.diag(np.diag(Mee))) == 0, "ECORR block not diagonal"
        out["mtcm_te"] = mtcm[np.ix_(tr, ec)]
        out["mtcm_ee_diag"] = np.diag(Mee).copy()
    # the T-block of the full inverse is the inverse of the Schur complement
    out["xvar_tr"] = xvar[np.ix_(tr, tr)]
    out["norm"] = norm
    # phiinv / norm^2 exactly as fitter.py:2166-2185 forms it
    phi = model.noise_model_basis_weight(toas)
    phiinv = np.zeros(ntm)
    if phi is not None:
        phiinv = np.concatenate((phiinv, 1 / phi))
    out["phiinv_n"] = phiinv / norm ** 2
    # column ranges of each noise component in the reference's mtcm ordering
    comps = sorted(dims.items(), key=lambda kv: kv[1][0])
    out["noise_comp_names"] = np.array([c for c, _ in comps])
    out["noise_comp_ranges"] = np.array([[d[0] + ntm, d[0] + ntm + d[1]] for _, d in comps], dtype=np.int64)
    out["ntm"] = np.array([ntm])
    out["gls_chi2_returned"] = np.array([float(chi2)])
    for k, v in f.resids.noise_resids.items():
        out["noise_resid_" + k] = np.asarray(v.to_value(u.s), dtype=np.float64)
    # the Woodbury chi2 of the reference's own post-fit residuals: what fit_toas returned
    # (residuals.py:567-589 on f.resids)
    out["post_resid"] = np.asarray(f.resids.time_resids.to_value(u.s), dtype=np.float64)
    c2, ln = f.resids.calc_chi2(lognorm=True)
    out["post_chi2"] = np.array([float(c2)])
    out["post_lognorm"] = np.array([float(ln)])
    # update_model (fitter.py:530-555) keywords written into the model
    um = {}
    for k in ("CHI2", "CHI2R", "TRES", "NTOA", "START", "FINISH", "DMDATA"):
        if hasattr(f.model, k):
            v = getattr(f.model, k).value
            um[k] = float(v) if v is not None and not isinstance(v, (bool, str)) else v
    out["update_model_keys"] = np.array(list(um.keys()))
    out["update_model_vals"] = np.array([np.nan if v is None else float(v) for v in um.values()])
    if name == "j0740":
        fit = pfit.GLSFitter(toas, copy.deepcopy(model))
        fit.fit_toas(maxiter=1)
        m2 = np.linspace(0.2, 0.3, 5)
        sini = np.sin(np.deg2rad(np.linspace(86.25, 88.5, 5)))
        out["grid_M2"], out["grid_SINI"] = m2, sini
        g = pfit.GLSFitter(toas, copy.deepcopy(fit.model))
        c_s, ex_s = grid_chisq(g, ("M2", "SINI"), (m2 * u.Msun, sini * u.dimensionless_unscaled),
                               extraparnames=["PB"], ncpu=1, printprogress=False)
        out["grid_chi2_serial"] = np.asarray(c_s, dtype=np.float64)
        g = pfit.GLSFitter(toas, copy.deepcopy(fit.model))
        c_p, ex_p = grid_chisq(g, ("M2", "SINI"), (m2 * u.Msun, sini * u.dimensionless_unscaled),
                               extraparnames=["PB"], ncpu=2, printprogress=False)
        out["grid_chi2_parallel"] = np.asarray(c_p, dtype=np.float64)
        pb = np.asarray([np.longdouble(getattr(x, "value", x)) for x in np.ravel(ex_p["PB"])], dtype=np.longdouble)
        h, l = split_ld(pb)
        out["grid_PB_parallel_hi"], out["grid_PB_parallel_lo"] = h.reshape(c_p.shape), l.reshape(c_p.shape)
        # the fitter the grid started from (its post-fit model is the grid's base model)
        out["grid_base_params"] = np.array(list(fit.model.free_params))
        vals = [split_ld(np.longdouble(getattr(fit.model, p).value)) for p in fit.model.free_params]
        out["grid_base_hi"] = np.array([v[0] for v in vals], dtype=np.float64)
        out["grid_base_lo"] = np.array([v[1] for v in vals], dtype=np.float64)
    path = os.path.join(GOLDEN, name + "_stage.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {os.path.getsize(path) / 1024:.1f} KiB, K={K}", file=sys.stderr)


if __name__ == "__main__":
    register_clockless_sites()
    for n in sys.argv[1:] or ["pta_iso", "pta_ell1", "pta_dd", "j0740", "b1855"]:
        stage(n)
