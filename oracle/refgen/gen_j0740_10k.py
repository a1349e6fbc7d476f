"""C3/C4 at a bench-like size (reference run; container only; TEST INFRASTRUCTURE).

J0740+6620 (the C3 model: ELL1 + Shapiro, ecliptic + PM, FD1, 68 DMX, EFAC/EQUAD/ECORR,
JUMP) on 10,000 synthetic TOAs by the same recipe as gen_synth.gen_j0740 (seed 0,
make_fake_toas_uniform 56640-58461, 820/1400 MHz alternating, 1 us, receivers by frequency,
re-zeroed with noise, empty DMX/JUMP masks frozen) -- ten times the j0740 fixture, the
size the reference fits here in ~26 s (bench/reference_cpu.json).

Recorded from the reference:
* the packed TOAs, masks and pre-fit residual outputs (no design matrix: 10k x K doubles);
* DownhillGLSFitter.fit_toas(maxiter=10) (fitter.py:1015-1105): status, chi2, fitted values
  (dd pairs), uncertainties;
* GLSFitter.fit_toas(maxiter=1): chi2, values, uncertainties, covariance, fac;
* a 16 x 16 patch of the bench's 256 x 256 (M2, SINI) grid (bench.py j0740_legs: M2 =
  linspace(0.2, 0.3, 256), SINI = sin(linspace(86.25, 88.5, 256) deg); indices 120..135 of
  each axis) with grid_chisq's parallel executor (ncpu=8; each point a deep copy of the
  GLSFitter the grid starts from, gridutils.py:72), chi2 and the extra parameter PB;
* the reference's own spread: the GLSFitter and DownhillGLSFitter fits rerun with every
  time residual shifted by a fixed per-TOA N(0, 5 ps) draw (seeds 1..NREP; as
  gen_downhill_spread.py), max |chi2 - chi2_0| / chi2_0, max |p - p_0| / sigma per
  parameter and max |corr - corr_0| of the GLS correlation matrix -- the floor that two
  longdouble / double-double evaluations of the same model differ by.

Usage: oracle/refenv/run_ref.sh oracle/refgen/gen_j0740_10k.py [--no-grid] [--no-spread]
Writes tests/golden/j0740_10k.{npz,json}.
"""
import copy
import os
import sys

import numpy as np
import astropy.units as u

from refcommon import (GOLDEN, register_clockless_sites, pack_toas, export_model, mask_table, residual_outputs,
                       split_ld, save)
import pint.fitter as pfit
import pint.residuals as pres
import pint.simulation as sim
from pint.gridutils import grid_chisq

import gen_synth

NTOA = 10000
GSIDE, G0, GN = 256, 120, 16
NREP = 4
SIGMA_S = 5e-12


def build():
    np.random.seed(0)
    model = gen_synth.j0740_model()
    ts = sim.make_fake_toas_uniform(56640, 58461, NTOA, model, freq=np.array([820, 1400]) * u.MHz,
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


def fit_gls(model, toas):
    f = pfit.GLSFitter(toas, copy.deepcopy(model))
    chi2 = float(f.fit_toas(maxiter=1))
    return f, chi2


def fit_down(model, toas):
    f = pfit.DownhillGLSFitter(toas, copy.deepcopy(model))
    try:
        f.fit_toas(maxiter=10)
        status = "converged"
    except Exception as e:  # MaxiterReached / StepProblem: recorded, as grid_chisq does
        status = type(e).__name__
    return f, status


def values(f):
    return {p: np.longdouble(getattr(f.model, p).value) for p in f.model.free_params}


def errors(f):
    return {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}


def spread(model, toas, g0, d0):
    """The reference's own spread under fixed per-TOA 5 ps residual shifts."""
    orig = pres.Residuals.calc_time_resids
    v0g, e0g, c0g = values(g0), errors(g0), float(g0.resids.chi2)
    corr0 = np.asarray(g0.parameter_correlation_matrix.matrix, dtype=np.float64)
    v0d, e0d, c0d = values(d0[0]), errors(d0[0]), float(d0[0].resids.chi2)
    out = {"gls_chi2_rel": 0.0, "gls_corr_abs": 0.0, "gls_err_rel": 0.0, "down_chi2_rel": 0.0,
           "gls_param_sigma": {p: 0.0 for p in v0g}, "down_param_sigma": {p: 0.0 for p in v0d},
           "down_status": [d0[1]], "nrep": NREP, "sigma_s": SIGMA_S}
    try:
        for rep in range(1, NREP + 1):
            shift = np.random.default_rng(rep).normal(0.0, SIGMA_S, toas.ntoas) * u.s

            def calc(self, *a, **k):
                return orig(self, *a, **k) + shift
            pres.Residuals.calc_time_resids = calc
            g, c = fit_gls(model, toas)
            out["gls_chi2_rel"] = max(out["gls_chi2_rel"], abs(float(g.resids.chi2) / c0g - 1))
            corr = np.asarray(g.parameter_correlation_matrix.matrix, dtype=np.float64)
            out["gls_corr_abs"] = max(out["gls_corr_abs"], float(np.max(np.abs(corr - corr0))))
            for p, v in values(g).items():
                out["gls_param_sigma"][p] = max(out["gls_param_sigma"][p], float(abs(v - v0g[p]) / e0g[p]))
                out["gls_err_rel"] = max(out["gls_err_rel"], abs(errors(g)[p] / e0g[p] - 1))
            d, st = fit_down(model, toas)
            out["down_status"].append(st)
            out["down_chi2_rel"] = max(out["down_chi2_rel"], abs(float(d.resids.chi2) / c0d - 1))
            for p, v in values(d).items():
                out["down_param_sigma"][p] = max(out["down_param_sigma"][p], float(abs(v - v0d[p]) / e0d[p]))
            print(f"spread rep {rep}: gls chi2 {out['gls_chi2_rel']:.2e} corr {out['gls_corr_abs']:.2e} "
                  f"down chi2 {out['down_chi2_rel']:.2e}", file=sys.stderr, flush=True)
    finally:
        pres.Residuals.calc_time_resids = orig
    return out


def gen(do_grid=True, do_spread=True):
    model, ts = build()
    arr, flags = pack_toas(ts)
    tz = model.get_TZR_toa(ts)
    tza, _ = pack_toas(tz)
    arrays = dict(arr)
    arrays.update({"tzr_" + k: v for k, v in tza.items()})
    arrays.update(mask_table(model, ts))
    _, ra, rm = residual_outputs(model, ts)
    arrays.update(ra)
    meta = {"name": "j0740_10k", "model": export_model(model), "flags": flags}
    obs = [str(o) for o in ts.get_obss()]
    meta["obs_names"] = sorted(set(obs))
    arrays["obs_index"] = np.array([meta["obs_names"].index(o) for o in obs], dtype=np.int16)
    meta.update(rm)
    g, chi2 = fit_gls(model, ts)
    meta["gls_chi2"] = chi2
    meta["gls_params"] = {p: list(map(float, split_ld(v))) for p, v in values(g).items()}
    meta["gls_errors"] = errors(g)
    arrays["gls_cov"] = np.asarray(g.parameter_covariance_matrix.matrix, dtype=np.float64)
    arrays["gls_corr"] = np.asarray(g.parameter_correlation_matrix.matrix, dtype=np.float64)
    arrays["gls_fac"] = np.asarray(g.fac, dtype=np.float64)
    print(f"GLS chi2 {chi2}", file=sys.stderr, flush=True)
    d, status = fit_down(model, ts)
    meta["down_status"] = status
    meta["down_chi2"] = float(d.resids.chi2)
    meta["down_params"] = {p: list(map(float, split_ld(v))) for p, v in values(d).items()}
    meta["down_errors"] = errors(d)
    print(f"Downhill {status} chi2 {meta['down_chi2']}", file=sys.stderr, flush=True)
    if do_grid:
        m2 = np.linspace(0.2, 0.3, GSIDE)[G0:G0 + GN]
        sini = np.sin(np.deg2rad(np.linspace(86.25, 88.5, GSIDE)))[G0:G0 + GN]
        gf = pfit.GLSFitter(ts, copy.deepcopy(g.model))
        c, ex = grid_chisq(gf, ("M2", "SINI"), (m2 * u.Msun, sini * u.dimensionless_unscaled),
                           extraparnames=["PB"], ncpu=8, printprogress=False)
        arrays["grid_M2"], arrays["grid_SINI"] = m2, sini
        arrays["grid_chi2"] = np.asarray(c, dtype=np.float64)
        pb = np.asarray([np.longdouble(getattr(x, "value", x)) for x in np.ravel(ex["PB"])], dtype=np.longdouble)
        h, l = split_ld(pb)
        arrays["grid_PB_hi"], arrays["grid_PB_lo"] = h.reshape(c.shape), l.reshape(c.shape)
        vals = [split_ld(np.longdouble(getattr(g.model, p).value)) for p in g.model.free_params]
        meta["grid_base_params"] = list(g.model.free_params)
        arrays["grid_base_hi"] = np.array([v[0] for v in vals], dtype=np.float64)
        arrays["grid_base_lo"] = np.array([v[1] for v in vals], dtype=np.float64)
        print(f"grid chi2 range {np.nanmin(c)} .. {np.nanmax(c)}", file=sys.stderr, flush=True)
    if do_spread:
        meta["spread"] = spread(model, ts, g, (d, status))
    save("j0740_10k", arrays, meta)


if __name__ == "__main__":
    register_clockless_sites()
    gen(do_grid="--no-grid" not in sys.argv, do_spread="--no-spread" not in sys.argv)
