"""PLANET_SHAPIRO fixtures (solar_system_shapiro.py:105-124, toa.py:2403-2433) -- reference
run, container only.

* planet_ngc   : NGC6440E with PLANET_SHAPIRO Y, TOAs loaded with planets=True (the model's
                 choice, toa.py:226-231): packed TOAs incl. obs_<planet>_pos, per-component
                 delays, phase, residuals, design matrix and one WLSFitter iteration.
* planet_b1855 : B1855+09 (9-yr, GLS) likewise, kept small: the Shapiro component, total
                 delay, residuals, the planet vectors on every 8th TOA and one GLSFitter
                 iteration (the device test prepares the TOAs from the tim file itself).
The par files are the reference's own with PLANET_SHAPIRO set to Y.
"""
import copy
import os

import numpy as np
import astropy.units as u

from refcommon import (GOLDEN, REFDATA, register_clockless_sites, pack_toas, export_model, mask_table,
                       component_delays, phase_outputs, residual_outputs, designmatrix_outputs,
                       split_ld, save)
import pint.toa as toa
from pint.models import get_model
from pint.fitter import WLSFitter, GLSFitter

PLANETS = ("jupiter", "saturn", "venus", "uranus", "neptune", "earth")


def planet_par(src, name):
    with open(f"{REFDATA}/{src}") as f:
        txt = f.read()
    lines = [ln for ln in txt.splitlines() if not ln.split()[:1] == ["PLANET_SHAPIRO"]]
    txt = "\n".join(lines) + "\nPLANET_SHAPIRO Y\n"
    path = os.path.join(GOLDEN, f"{name}.par")
    with open(path, "w") as f:
        f.write(txt)
    return path


def fit_meta(f, key):
    return {f"{key}_chi2": float(f.resids.chi2),
            f"{key}_params": {p: list(map(float, split_ld(getattr(f.model, p).value))) for p in f.model.free_params},
            f"{key}_errors": {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}}


def main():
    register_clockless_sites()
    # NGC6440E
    par = planet_par("NGC6440E.par", "planet_ngc")
    model = get_model(par)
    assert model.PLANET_SHAPIRO.value
    toas = toa.get_TOAs(f"{REFDATA}/NGC6440E.tim", ephem="builtin", include_bipm=False, model=model)
    assert toas.planets
    arr, flags = pack_toas(toas)
    tz = model.get_TZR_toa(toas)
    tza, _ = pack_toas(tz)
    arrays = dict(arr)
    arrays.update({"tzr_" + k: v for k, v in tza.items()})
    arrays.update(mask_table(model, toas))
    arrays.update(component_delays(model, toas))
    arrays.update(phase_outputs(model, toas))
    r, ra, rm = residual_outputs(model, toas)
    arrays.update(ra)
    dm, dmm = designmatrix_outputs(model, toas)
    arrays.update(dm)
    meta = {"name": "planet_ngc", "model": export_model(model), "flags": flags}
    meta.update(rm)
    meta.update(dmm)
    f = WLSFitter(toas, copy.deepcopy(model))
    f.fit_toas(maxiter=1)
    meta.update(fit_meta(f, "wls"))
    arrays["wls_post_resid"] = np.asarray(f.resids.time_resids.to_value(u.s))
    save("planet_ngc", arrays, meta)

    # B1855+09
    par = planet_par("B1855+09_NANOGrav_9yv1.gls.par", "planet_b1855")
    model = get_model(par)
    toas = toa.get_TOAs(f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", ephem="builtin", include_bipm=False,
                        model=model)
    assert toas.planets
    rows = np.arange(0, toas.ntoas, 8)
    arrays = {"rows": rows}
    arr, _ = pack_toas(toas)
    for pl in PLANETS:
        arrays[f"obs_{pl}_pos_km"] = arr[f"obs_{pl}_pos_km"][rows]
    cd = component_delays(model, toas)
    arrays["delay_total"] = cd["delay_total"]
    arrays.update({k: v for k, v in cd.items() if "shapiro" in k.lower() and "binary" not in k.lower()})
    r, ra, rm = residual_outputs(model, toas)
    arrays["res_time"] = ra["res_time"]
    meta = {"name": "planet_b1855", "model": export_model(model)}
    meta.update(rm)
    f = GLSFitter(toas, copy.deepcopy(model))
    f.fit_toas(maxiter=1)
    meta.update(fit_meta(f, "gls"))
    save("planet_b1855", arrays, meta)


if __name__ == "__main__":
    main()
