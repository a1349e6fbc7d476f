"""Golden fixture C2: B1855+09 NANOGrav 9-yr (DD, ecliptic+PM, FD1-3, DMX, JUMP,
EFAC/EQUAD, ECORR, PLRedNoise) — reference run on the offline recipe (container only).

Full 4005 TOAs are packed; the design matrix is stored on every 8th row only to keep
the fixture small (fixtures <= ~1 MB).
"""
import copy

import numpy as np
import astropy.units as u

from refcommon import (REFDATA, register_clockless_sites, pack_toas, export_model, mask_table,
                       component_delays, phase_outputs, residual_outputs, designmatrix_outputs,
                       noise_outputs, split_ld, save)
import pint.toa as toa
from pint.models import get_model
from pint.fitter import GLSFitter


def main():
    register_clockless_sites()
    model = get_model(f"{REFDATA}/B1855+09_NANOGrav_9yv1.gls.par")
    toas = toa.get_TOAs(f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", ephem="builtin",
                        include_bipm=False, planets=False, model=model)
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
    rows = np.arange(0, toas.ntoas, 8)
    arrays["dm_rows"] = rows
    arrays["dm_M"] = dm["dm_M"][rows]
    no, nm = noise_outputs(model, toas)
    arrays.update(no)
    arrays["psr_dir_icrs"] = np.asarray(model.ssb_to_psb_xyz_ICRS(
        epoch=toas.table["tdbld"].astype(np.float64)), dtype=np.float64)
    meta = {"name": "b1855", "model": export_model(model), "flags": flags}
    meta.update(rm)
    meta.update(dmm)
    meta.update(nm)
    f = GLSFitter(toas, copy.deepcopy(model))
    chi2 = f.fit_toas(maxiter=1)
    meta["gls_chi2"] = float(chi2)
    meta["gls_params"] = {p: list(map(float, split_ld(getattr(f.model, p).value)))
                          for p in f.model.free_params}
    meta["gls_errors"] = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
    ntm = len(f.model.free_params) + 1
    arrays["gls_cov"] = np.asarray(f.parameter_covariance_matrix.matrix, dtype=np.float64)[:ntm, :ntm]
    arrays["gls_fac"] = np.asarray(f.fac, dtype=np.float64)
    arrays["gls_post_resid"] = np.asarray(f.resids.time_resids.to_value(u.s))
    save("b1855", arrays, meta)


if __name__ == "__main__":
    main()
