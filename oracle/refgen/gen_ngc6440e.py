"""Golden fixture C1: NGC6440E (isolated, equatorial, DM) — reference run (container only).

Captures packed TOAs, model table, per-component delays, phase, residuals, design
matrix, one WLSFitter iteration, a DownhillWLS fit and a 5x5 (F0,F1) grid_chisq
(serial warm-start and parallel cold-start), per SURVEY.md §8(c) "Fixtures to capture".
"""
import copy
import sys

import numpy as np
import astropy.units as u

from refcommon import (REFDATA, register_clockless_sites, pack_toas, export_model, mask_table,
                       component_delays, phase_outputs, residual_outputs, designmatrix_outputs,
                       split_ld, save)
import pint.toa as toa
from pint.models import get_model
from pint.fitter import WLSFitter, DownhillWLSFitter
from pint.gridutils import grid_chisq


def main():
    register_clockless_sites()
    model = get_model(f"{REFDATA}/NGC6440E.par")
    toas = toa.get_TOAs(f"{REFDATA}/NGC6440E.tim", ephem="builtin", include_bipm=False,
                        planets=False, model=model)
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
    meta = {"name": "ngc6440e", "model": export_model(model), "flags": flags}
    meta.update(rm)
    meta.update(dmm)

    # one WLS iteration (fitter.py:1965)
    f = WLSFitter(toas, model)
    chi2 = f.fit_toas(maxiter=1)
    meta["wls_chi2"] = float(chi2)
    meta["wls_params"] = {p: list(map(float, split_ld(getattr(f.model, p).value))) for p in f.model.free_params}
    meta["wls_errors"] = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
    arrays["wls_cov"] = np.asarray(f.parameter_covariance_matrix.matrix, dtype=np.float64)
    arrays["wls_post_resid"] = np.asarray(f.resids.time_resids.to_value(u.s))

    # downhill WLS (fitter.py:1379)
    fd = DownhillWLSFitter(toas, model)
    fd.fit_toas(maxiter=10)
    meta["dwls_chi2"] = float(fd.resids.chi2)
    meta["dwls_converged"] = bool(fd.converged)
    meta["dwls_params"] = {p: list(map(float, split_ld(getattr(fd.model, p).value))) for p in fd.model.free_params}
    meta["dwls_errors"] = {p: float(getattr(fd.model, p).uncertainty_value) for p in fd.model.free_params}

    # grid_chisq (gridutils.py:166) over (F0, F1) +-3 sigma of the WLS best fit
    F0 = f.model.F0.value
    F1 = f.model.F1.value
    sF0 = f.model.F0.uncertainty_value
    sF1 = f.model.F1.uncertainty_value
    g0 = np.longdouble(F0) + np.linspace(-3, 3, 5) * np.longdouble(sF0)
    g1 = np.longdouble(F1) + np.linspace(-3, 3, 5) * np.longdouble(sF1)
    gh0, gl0 = split_ld(g0)
    gh1, gl1 = split_ld(g1)
    arrays.update(grid_F0_hi=gh0, grid_F0_lo=gl0, grid_F1_hi=gh1, grid_F1_lo=gl1)
    fg = WLSFitter(toas, copy.deepcopy(f.model))
    chi2s, _ = grid_chisq(fg, ("F0", "F1"), (g0 * u.Hz, g1 * u.Hz / u.s), ncpu=1, printprogress=False)
    arrays["grid_chi2_serial"] = np.asarray(chi2s, dtype=np.float64)
    fg = WLSFitter(toas, copy.deepcopy(f.model))
    chi2p, _ = grid_chisq(fg, ("F0", "F1"), (g0 * u.Hz, g1 * u.Hz / u.s), ncpu=2, printprogress=False)
    arrays["grid_chi2_parallel"] = np.asarray(chi2p, dtype=np.float64)
    save("ngc6440e", arrays, meta)


if __name__ == "__main__":
    main()
