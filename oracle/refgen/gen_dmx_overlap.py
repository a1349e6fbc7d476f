"""Overlapping DMX bins (dispersion_model.py:659-708: every bin whose [DMXR1, DMXR2] holds a
TOA adds its DMX_ to that TOA's DM and has a 1 in its design-matrix column) -- reference run,
container only.  NGC6440E with six free DMX bins, some TOAs in 3 and 4 bins at once
(53801-53843: bins 2, 3, 4; 53833: bins 2, 3, 4, 5), six TOAs in none (DM stays determined).
Captures the packed TOAs, per-component delays, residuals, design matrix and one WLSFitter
iteration -> tests/golden/dmx_overlap.{npz,json,par}."""
import copy
import os

import numpy as np
import astropy.units as u

from refcommon import (GOLDEN, REFDATA, register_clockless_sites, pack_toas, export_model, mask_table,
                       component_delays, phase_outputs, residual_outputs, designmatrix_outputs,
                       split_ld, save)
import pint.toa as toa
from pint.models import get_model
from pint.fitter import WLSFitter

BINS = [(1, 0.0012, 53670.0, 53760.0), (2, -0.0021, 53700.0, 53900.0), (3, 0.0017, 53730.0, 54020.0),
        (4, 0.0006, 53800.0, 53850.0), (5, -0.0009, 53830.0, 53840.0), (6, 0.0004, 54090.0, 54160.0)]


def main():
    register_clockless_sites()
    with open(f"{REFDATA}/NGC6440E.par") as f:
        txt = f.read().rstrip("\n") + "\n"
    txt += "DMX 14.0\n"
    for k, v, r1, r2 in BINS:
        txt += f"DMX_{k:04d} {v} 1\nDMXR1_{k:04d} {r1}\nDMXR2_{k:04d} {r2}\n"
    par = os.path.join(GOLDEN, "dmx_overlap.par")
    with open(par, "w") as f:
        f.write(txt)
    model = get_model(par)
    toas = toa.get_TOAs(f"{REFDATA}/NGC6440E.tim", ephem="builtin", include_bipm=False, planets=False,
                        model=model)
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
    arrays["dmx_dm"] = np.asarray(model.dmx_dm(toas).to_value(u.pc / u.cm ** 3), dtype=np.float64)
    meta = {"name": "dmx_overlap", "model": export_model(model), "flags": flags}
    meta.update(rm)
    meta.update(dmm)
    f = WLSFitter(toas, copy.deepcopy(model))
    f.fit_toas(maxiter=1)
    meta["wls_chi2"] = float(f.resids.chi2)
    meta["wls_params"] = {p: list(map(float, split_ld(getattr(f.model, p).value))) for p in f.model.free_params}
    meta["wls_errors"] = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
    arrays["wls_post_resid"] = np.asarray(f.resids.time_resids.to_value(u.s))
    save("dmx_overlap", arrays, meta)


if __name__ == "__main__":
    main()
