"""Helpers to load the committed golden fixtures (test infrastructure)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PARS = {"ngc6440e": "NGC6440E.par", "b1855": "B1855+09_NANOGrav_9yv1.gls.par", "j0740": "J0740+6620.par",
        "pta_iso": "pta_iso.par", "pta_ell1": "pta_ell1.par", "pta_dd": "pta_dd.par",
        "wls_phoff": "wls_phoff.par", "ecorr_phoff": "ecorr_phoff.par", "wls_noise": "wls_noise.par",
        "ecorr_fit": "ecorr_fit.par", "white_mjd": "white_mjd.par", "ell1h_h3": "ell1h_h3.par",
        "ell1h_h4": "ell1h_h4.par", "ell1h_stig": "ell1h_stig.par", "pta_bt": "pta_bt.par",
        "pta_dmn": "pta_dmn.par", "pta_ddk": "pta_ddk.par", "pta_ddk_nk": "pta_ddk_nk.par",
        "wb_dd": "wb_dd.par", "c5_iso": "c5_iso.par", "c5_ell1": "c5_ell1.par", "c5_dd": "c5_dd.par",
        "planet_ngc": "planet_ngc.par", "planet_b1855": "planet_b1855.par",
        "dmx_overlap": "dmx_overlap.par", "j0740_10k": "J0740+6620.par",
        "phoff_red": "phoff_red.par", "phoff_ecorr": "phoff_ecorr.par", "phoff_dmn": "phoff_dmn.par"}


def load(name):
    from pint_amd import get_model
    from pint_amd.toa import from_arrays_with_tzr
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    fc = dict(meta["flag_columns"])
    if "wb_pp_dm" in z:  # the wideband -pp_dm / -pp_dme flags, as the tim file carries them
        fc["pp_dm"] = [repr(float(x)) for x in z["wb_pp_dm"]]
        fc["pp_dme"] = [repr(float(x)) for x in z["wb_pp_dme"]]
    toas = from_arrays_with_tzr(z, fc, name, meta.get("obs_names"))
    model = get_model(os.path.join(GOLDEN, PARS[name]))
    free = [p for p in meta["model"]["free_params"]]
    model.free_params = [p for p in free if p in model]
    return model, toas, z, meta


def ref_value(meta, key, p):
    v = meta[key][p]
    return np.longdouble(v[0]) + np.longdouble(v[1])


def downhill_bar(name, p, floor=1e-3):
    """Per-parameter Downhill bar (sigma units): 2x the reference's own spread when its
    residuals are perturbed at the 5 ps longdouble floor (tests/golden/downhill_spread.json,
    oracle/refgen/gen_downhill_spread.py), at least `floor` (1e-3 sigma)."""
    d = json.load(open(os.path.join(GOLDEN, "downhill_spread.json")))
    if name not in d:
        return floor
    return max(floor, 2.0 * d[name]["max_dev_sigma"].get(p, 0.0))


_SPREAD = None
SPREAD_MAX_PS = 30.0  # the largest residual shift oracle/refgen/gen_fit_spread.py measured


def rms_ps(a, b) -> float:
    """rms of the difference of two time-residual arrays (s), in ps."""
    return float(np.sqrt(np.mean((np.asarray(a, dtype=np.float64) - np.asarray(b, dtype=np.float64)) ** 2)) * 1e12)


def chi2_bar(name, kind, resid_rms_ps, floor=1e-9):
    """End-to-end relative chi2 bar of fixture `name` (kind "pre": the pre-fit Residuals chi2,
    "fit": the GLSFitter / WLSFitter fit_toas(maxiter=1) chi2, "down": the DownhillGLSFitter
    chi2): 2x the reference's own chi2 spread when its time residuals move by as much as the
    residuals under test differ from the reference's.  tests/golden/fit_spread.json
    (oracle/refgen/gen_fit_spread.py) holds max |chi2 / chi2_0 - 1| of the reference under fixed
    per-TOA N(0, 5 ps) and N(0, 30 ps) residual shifts; the bar scales the larger per-ps rate
    to the measured rms difference `resid_rms_ps` (at least the 5 ps longdouble floor).

    The spread is calibrated over 5-30 ps of residual difference, so the bar stops widening at
    SPREAD_MAX_PS: a residual drift beyond it must move chi2 inside the calibrated bar or fail,
    not widen its own bar."""
    global _SPREAD
    if _SPREAD is None:
        _SPREAD = json.load(open(os.path.join(GOLDEN, "fit_spread.json")))
    d = _SPREAD[name]
    per_ps = max(d["5ps"][kind] / 5.0, d["30ps"][kind] / 30.0)
    return max(floor, 2.0 * per_ps * min(max(float(resid_rms_ps), 5.0), SPREAD_MAX_PS))


def grid_tables(lay, grid):
    """The point tables pint_set_grid forms on the device (k_grid_tables), restated on the
    host: grid = (base table, [(name, values, stride, size)], npts, k0); point k takes
    values[((k0 + k) // stride) % size] as a (hi, lo) pair."""
    base, variables, npts, k0 = grid
    tabs = np.tile(np.asarray(base, dtype=np.float64), (npts, 1))
    k = np.arange(npts, dtype=np.int64) + int(k0)
    for name, vals, stride, size in variables:
        v = np.asarray(vals, dtype=np.longdouble).reshape(-1)[(k // int(stride)) % int(size)]
        h = v.astype(np.float64)
        o = lay.offsets[name]
        tabs[:, o] = h
        tabs[:, o + 1] = (v - h.astype(np.longdouble)).astype(np.float64)
    return tabs
