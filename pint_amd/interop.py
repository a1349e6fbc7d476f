"""The drop-in boundary from PINT objects: a reference ``pint.models.TimingModel`` and
``pint.toa.TOAs`` (with the TZR TOA of ``AbsPhase.get_TZR_toa``) into pint_amd's host
objects, and fitted values back into the PINT model.

A PINT user keeps loading data the reference's way -- ``get_model_and_toas(par, tim)``
(/root/reference/src/pint/models/model_builder.py:859), clock corrections, TDB and
ephemeris lookup on the host (toa.py:2251 compute_TDBs, :2323 compute_posvels) -- and hands
the result to the GPU path once:

    pm, pt = interop.from_pint(model, toas)     # packed per-TOA columns + parameter table
    f = pint_amd.GLSFitter(pt, pm)              # same fitter API as pint.fitter
    f.fit_toas()
    interop.update_pint_model(f.model, model)   # fitted values/uncertainties -> PINT model

Nothing here imports PINT at module load: the functions take the PINT objects as
arguments and read only their public attributes, so pint_amd itself needs neither PINT nor
astropy (the GPU box has neither).

What is read (the columns the reference's own model evaluation reads):
* TOAs.table: ``tdbld`` (longdouble -> exact double-double split), ``freq`` (MHz),
  ``error`` (us), ``ssb_obs_pos`` (km), ``ssb_obs_vel`` (km/s), ``obs_sun_pos`` (km),
  ``mjd_float``, ``obs`` (barycentric flag), ``pulse_number``, ``delta_pulse_number``
  and the flag dicts (toa.py:2320-2489);
* the TZR TOA the reference builds (models/absolute_phase.py:79-127 get_TZR_toa), packed
  the same way;
* the model: its structure through its own par-file text (timing_model.py:2747
  as_parfile), then every parameter's value, frozen flag and uncertainty from the
  parameter objects themselves -- MJD parameters through their astropy Time at full
  precision (pulsar_mjd.py:286 time_to_longdouble), long-double parameters unrounded.
"""
from __future__ import annotations

import numpy as np

from .parameter import LD
from .toa import TOAs


def _q(col, unit):
    """A table column in `unit` as float64, whether it is a Quantity column or plain."""
    try:
        return np.asarray(col.quantity.to_value(unit), dtype=np.float64)
    except AttributeError:
        return np.asarray(col.to_value(unit) if hasattr(col, "to_value") else col, dtype=np.float64)


def _split(x):
    x = np.asarray(x, dtype=np.longdouble)
    hi = x.astype(np.float64)
    return hi, (x - hi.astype(np.longdouble)).astype(np.float64)


def pack_pint_toas(toas):
    """(arrays, flags) of a PINT TOAs object in pint_amd's boundary schema."""
    import astropy.units as u
    t = toas.table
    hi, lo = _split(t["tdbld"])
    out = {
        "tdb_hi": hi, "tdb_lo": lo,
        "freq_mhz": _q(t["freq"], u.MHz),
        "err_us": _q(t["error"], u.us),
        "ssb_obs_pos_km": _q(t["ssb_obs_pos"], u.km),
        "ssb_obs_vel_kms": _q(t["ssb_obs_vel"], u.km / u.s),
        "obs_sun_pos_km": _q(t["obs_sun_pos"], u.km),
        "mjd_float": np.asarray(t["mjd_float"], dtype=np.float64),
        "is_bary": np.asarray(toas.get_obss() == "barycenter", dtype=np.uint8),
    }
    if "pulse_number" in t.colnames:
        out["pulse_number"] = np.asarray(t["pulse_number"], dtype=np.float64)
    out["delta_pulse_number"] = (np.asarray(t["delta_pulse_number"], dtype=np.float64)
                                 if "delta_pulse_number" in t.colnames else np.zeros(len(t)))
    if "ssb_obs_vel_ecl" in t.colnames:
        out["ssb_obs_vel_ecl_kms"] = _q(t["ssb_obs_vel_ecl"], u.km / u.s)
    return out, [dict(f) for f in t["flags"]]


def toas_from_pint(toas, model=None) -> TOAs:
    """pint_amd TOAs from PINT TOAs (+ the model's TZR TOA when the model has AbsPhase or
    is given, as TimingModel.phase(abs_phase=True) uses it)."""
    arr, flags = pack_pint_toas(toas)
    keys = sorted({k for f in flags for k in f})
    fl = {k: [str(f.get(k, "")) for f in flags] for k in keys}
    tzr = None
    if model is not None and hasattr(model, "get_TZR_toa"):
        tz = model.get_TZR_toa(toas)
        ta, tf = pack_pint_toas(tz)
        tzr = {k: v for k, v in ta.items()}
        tzr["flags"] = {k: str(v) for k, v in tf[0].items()}
    name = str(getattr(model, "PSR", None).value) if model is not None and hasattr(model, "PSR") else ""
    out = TOAs(arr, fl, tzr, name)
    out.ephem = getattr(toas, "ephem", None)
    try:
        info = toas.clock_corr_info
        out.clock = f"TT({info['bipm_version']})" if info.get("include_bipm") else "TT(TAI)"
    except Exception:
        out.clock = None
    return out


def _pint_value(par):
    """A PINT parameter's value in par-file units at the precision the reference keeps."""
    from pint.models.parameter import AngleParameter, MJDParameter, boolParameter, strParameter
    if par.value is None:
        return None
    if isinstance(par, (strParameter, boolParameter)):
        return par.value
    if isinstance(par, MJDParameter):
        from pint.pulsar_mjd import time_to_longdouble
        return np.longdouble(time_to_longdouble(par.quantity))
    if isinstance(par, AngleParameter):
        return float(par.quantity.value)
    v = par.value
    return np.longdouble(v) if isinstance(v, np.longdouble) else v


def model_from_pint(model):
    """pint_amd TimingModel from a PINT TimingModel."""
    from .timing_model import get_model
    text = model.as_parfile(include_info=False)
    pm = get_model(text)
    for name in model.params:
        if name not in pm:
            continue
        par = getattr(model, name)
        ours = pm[name]
        if ours.kind in ("str", "bool"):
            continue
        v = _pint_value(par)
        if v is not None:
            if ours.kind == "mjd" or ours.long_double:
                ours.value = LD(v)
            elif ours.kind == "int":
                ours.value = int(v)
            else:
                ours.value = float(v)
        ours.frozen = bool(par.frozen)
        unc = getattr(par, "uncertainty_value", None)
        ours.uncertainty = None if unc is None else float(unc)
    pm.validate()
    return pm


def from_pint(model, toas):
    """(pint_amd TimingModel, pint_amd TOAs) of a PINT (TimingModel, TOAs) pair."""
    return model_from_pint(model), toas_from_pint(toas, model)


def update_pint_model(pm, model):
    """Write pint_amd's fitted values and uncertainties (and update_model's keywords) back
    into the PINT model, parameter by parameter, at full precision."""
    from pint.models.parameter import AngleParameter, MJDParameter, boolParameter, strParameter
    import astropy.units as u
    for name in model.params:
        if name not in pm:
            continue
        par = getattr(model, name)
        ours = pm[name]
        if isinstance(par, (strParameter, boolParameter)) or ours.value is None:
            continue
        if isinstance(par, MJDParameter):
            from astropy.time import Time
            day = np.floor(LD(ours.value))
            frac = LD(ours.value) - day
            par.quantity = Time(float(day), float(frac), format="pulsar_mjd", scale=par.quantity.scale
                                if par.quantity is not None else "tdb", precision=9)
        elif isinstance(par, AngleParameter):
            par.quantity = float(ours.value) * par.quantity.unit
        else:
            par.value = ours.value
        if ours.uncertainty is not None and not par.frozen:
            par.uncertainty_value = ours.uncertainty
    return model
