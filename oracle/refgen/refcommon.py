"""Shared helpers for the golden-fixture generators (TEST INFRASTRUCTURE ONLY).

These scripts import the read-only reference (PINT @ /root/reference/src) under
/opt/conda/bin/python3.9 via ``oracle/refenv/run_ref.sh`` and write small fixtures
into ``tests/golden/``.  They run only in the build container; nothing here is
imported by the product package, and nothing here travels to the GPU box except the
fixtures it writes (data: inputs and expected outputs).

Offline recipe: ephem="builtin" (erfa epv00), no clock
files (topocentric sites re-registered with apply_gps2utc=False and no clock file),
include_bipm=False.
"""
import json
import os
import sys
import warnings

import numpy as np

warnings.filterwarnings("ignore")

import astropy.units as u  # noqa: E402
import pint  # noqa: E402
import pint.config  # noqa: E402
import pint.toa as toa  # noqa: E402
from pint.models import get_model  # noqa: E402
from pint.observatory.topo_obs import TopoObs  # noqa: E402

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
REFDATA = "/root/reference/tests/datafile"
REFPROF = "/root/reference/profiling"

_SITES = {
    "gbt": dict(tempo_code="1", itoa_code="GB", aliases=["gb"]),
    "arecibo": dict(tempo_code="3", itoa_code="AO", aliases=["aoutc", "ao"]),
}


def register_clockless_sites():
    """Re-register topocentric sites without clock files (pint observatory API,
    ``observatory/topo_obs.py:139``) so TOAs load offline."""
    obs = json.load(open(os.path.join(os.path.dirname(pint.config.runtimefile("observatories.json")),
                                      "observatories.json")))
    for name, kw in _SITES.items():
        TopoObs(name, itrf_xyz=obs[name]["itrf_xyz"], apply_gps2utc=False, overwrite=True,
                clock_file="", **kw)


def split_ld(x):
    """Exact split of numpy longdouble into (hi, lo) float64 pair."""
    x = np.asarray(x, dtype=np.longdouble)
    hi = x.astype(np.float64)
    lo = (x - hi.astype(np.longdouble)).astype(np.float64)
    return hi, lo


def pack_toas(toas, model=None):
    """Pack a TOAs table into the SoA boundary schema."""
    t = toas.table
    hi, lo = split_ld(t["tdbld"])
    out = {
        "tdb_hi": hi,
        "tdb_lo": lo,
        "freq_mhz": np.asarray(t["freq"].quantity.to_value(u.MHz), dtype=np.float64),
        "err_us": np.asarray(t["error"].quantity.to_value(u.us), dtype=np.float64),
        "ssb_obs_pos_km": np.asarray(t["ssb_obs_pos"].quantity.to_value(u.km), dtype=np.float64),
        "ssb_obs_vel_kms": np.asarray(t["ssb_obs_vel"].quantity.to_value(u.km / u.s), dtype=np.float64),
        "obs_sun_pos_km": np.asarray(t["obs_sun_pos"].quantity.to_value(u.km), dtype=np.float64),
        "mjd_float": np.asarray(t["mjd_float"], dtype=np.float64),
        "is_bary": np.asarray(toas.get_obss() == "barycenter", dtype=np.uint8),
    }
    if "pulse_number" in t.colnames:
        out["pulse_number"] = np.asarray(t["pulse_number"], dtype=np.float64)
    if "delta_pulse_number" in t.colnames:
        out["delta_pulse_number"] = np.asarray(t["delta_pulse_number"], dtype=np.float64)
    else:
        out["delta_pulse_number"] = np.zeros(len(t))
    for pl in ("jupiter", "saturn", "venus", "uranus", "neptune", "earth"):   # planets=True (toa.py:2403)
        if f"obs_{pl}_pos" in t.colnames:
            out[f"obs_{pl}_pos_km"] = np.asarray(t[f"obs_{pl}_pos"].quantity.to_value(u.km), dtype=np.float64)
    if "ssb_obs_vel_ecl" in t.colnames:
        out["ssb_obs_vel_ecl_kms"] = np.asarray(t["ssb_obs_vel_ecl"].quantity.to_value(u.km / u.s),
                                                dtype=np.float64)
    flags = [dict(f) for f in t["flags"]]
    return out, flags


def ld_str(v):
    return np.format_float_positional(np.longdouble(v), unique=True, trim="-") if v is not None else None


def export_model(model):
    """Parameter table: name -> {value (hi/lo), units, frozen, kind, key/key_value}."""
    from pint.models.parameter import (MJDParameter, AngleParameter, boolParameter, strParameter,
                                       maskParameter, intParameter)
    rec = {}
    for p in model.params:
        par = getattr(model, p)
        d = {"frozen": bool(par.frozen), "units": str(par.units), "kind": type(par).__name__}
        v = par.value
        if isinstance(par, (strParameter, boolParameter)):
            d["value"] = None if v is None else str(v)
        elif v is None:
            d["value"] = None
        else:
            if isinstance(par, MJDParameter):
                vv = np.longdouble(par.value)
            elif isinstance(par, AngleParameter):
                vv = np.longdouble(par.quantity.value)
            else:
                try:
                    vv = np.longdouble(v)
                except Exception:
                    d["value"] = str(v)
                    rec[p] = d
                    continue
            hi, lo = split_ld(vv)
            d["value"] = [float(hi), float(lo)]
        if isinstance(par, maskParameter):
            d["key"] = par.key
            d["key_value"] = [str(x) for x in par.key_value] if par.key_value is not None else None
        if par.uncertainty is not None:
            try:
                d["uncertainty"] = float(par.uncertainty_value)
            except Exception:
                pass
        rec[p] = d
    comps = list(model.components.keys())
    return {"params": list(model.params), "values": rec, "components": comps,
            "free_params": list(model.free_params),
            "delay_components": [c.__class__.__name__ for c in model.DelayComponent_list],
            "phase_components": [c.__class__.__name__ for c in model.PhaseComponent_list]}


def mask_table(model, toas):
    """Per-TOA selection of each mask parameter (parameter.py:2124 select_toa_mask)."""
    from pint.models.parameter import maskParameter
    out = {}
    for p in model.params:
        par = getattr(model, p)
        if isinstance(par, maskParameter) and par.key is not None:
            m = np.zeros(toas.ntoas, dtype=np.uint8)
            m[par.select_toa_mask(toas)] = 1
            out["mask_" + p] = m
    return out


def component_delays(model, toas):
    """Each delay function's contribution, accumulated exactly as TimingModel.delay
    (timing_model.py:1515-1546)."""
    delay = np.zeros(toas.ntoas) * u.s
    parts = {}
    for dc in model.DelayComponent_list:
        for df in dc.delay_funcs_component:
            d = df(toas, delay)
            parts["delay_" + df.__name__] = np.asarray(d.to_value(u.s), dtype=np.float64)
            delay += d
    parts["delay_total"] = np.asarray(delay.to_value(u.s), dtype=np.float64)
    return parts


def phase_outputs(model, toas):
    out = {}
    ph = model.phase(toas, abs_phase=True)
    out["phase_int"] = np.asarray(ph.int.value, dtype=np.float64)
    fh, fl = split_ld(ph.frac.value)
    out["phase_frac_hi"], out["phase_frac_lo"] = fh, fl
    ph0 = model.phase(toas, abs_phase=False)
    out["phase_noabs_int"] = np.asarray(ph0.int.value, dtype=np.float64)
    out["phase_noabs_frac"] = np.asarray(ph0.frac.value, dtype=np.float64)
    tz = model.get_TZR_toa(toas)
    out["tzr_delay"] = np.asarray(model.delay(tz).to_value(u.s), dtype=np.float64)
    return out


def residual_outputs(model, toas, prefix="res_"):
    from pint.residuals import Residuals
    r = Residuals(toas, model)
    out = {
        prefix + "time": np.asarray(r.time_resids.to_value(u.s), dtype=np.float64),
        prefix + "phase": np.asarray(r.phase_resids.value, dtype=np.float64),
        prefix + "sigma_us": np.asarray(r.get_data_error().to_value(u.us), dtype=np.float64),
    }
    meta = {prefix + "chi2": float(r.chi2), prefix + "track_mode": r.track_mode,
            prefix + "dof": int(r.dof)}
    try:
        c2, ln = r.calc_chi2(lognorm=True)
        meta[prefix + "lognorm"] = float(ln)
        meta[prefix + "lnlikelihood"] = float(r.lnlikelihood())
    except Exception:
        pass
    meta[prefix + "rms_weighted_us"] = float(r.rms_weighted().to_value(u.us))
    return r, out, meta


def designmatrix_outputs(model, toas):
    M, params, units = model.designmatrix(toas)
    return {"dm_M": np.asarray(M, dtype=np.float64)}, {"dm_params": list(params),
                                                        "dm_units": [str(x) for x in units]}


def noise_outputs(model, toas):
    out = {}
    if model.has_correlated_errors:
        U = model.noise_model_designmatrix(toas)
        w = model.noise_model_basis_weight(toas)
        out["noise_U_ncols"] = np.array([U.shape[1]])
        out["noise_weights"] = np.asarray(w, dtype=np.float64)
        dims = model.noise_model_dimensions(toas)
        return out, {"noise_dims": {k: [int(a), int(b)] for k, (a, b) in dims.items()}}
    return out, {}


def compact_flags(meta):
    """Keep only the flag keys that mask parameters select on, column-wise."""
    keys = set()
    for d in meta["model"]["values"].values():
        if d.get("key"):
            keys.add(d["key"].lstrip("-"))
    flags = meta.pop("flags")
    meta["flag_columns"] = {k: [f.get(k, "") for f in flags] for k in sorted(keys)}


def save(name, arrays, meta):
    os.makedirs(GOLDEN, exist_ok=True)
    if "flags" in meta:
        compact_flags(meta)
    np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), **arrays)
    with open(os.path.join(GOLDEN, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True, default=str)
    sz = os.path.getsize(os.path.join(GOLDEN, name + ".npz"))
    print(f"wrote {name}: {sz/1024:.1f} KiB npz", file=sys.stderr)
