"""Golden fixture for the wideband DM residuals (reference run; container only).

* wb_dd : the C5 per-pulsar template with a DD binary (gen_synth.pta_par) plus DMJUMP,
          DMEFAC and DMEQUAD on MJD ranges; make_fake_toas_uniform(wideband=True) gives each
          TOA a -pp_dm / -pp_dme measurement (simulation.py update_fake_dms).  Captures the
          packed TOAs, the pp_dm / pp_dme columns, the reference's TOA residuals,
          WidebandDMResiduals (residuals.py:908: total_dm, scaled DM errors, resids, chi2,
          dof, rms_weighted) and WidebandTOAResiduals (its chi2 through WidebandTOAFitter
          with no free parameters, dof, reduced_chi2).
Usage: run_ref.sh gen_wideband.py
"""
import io

import numpy as np
import astropy.units as u

from refcommon import (register_clockless_sites, pack_toas, export_model, mask_table, component_delays,
                       phase_outputs, residual_outputs, noise_outputs, save, GOLDEN)
import pint.simulation as sim
from pint.models import get_model
from pint.residuals import Residuals, WidebandDMResiduals, WidebandTOAResiduals
from pint.fitter import WidebandTOAFitter, WidebandDownhillFitter
from refcommon import split_ld
import copy
from gen_synth import pta_par

EXTRA = """DMJUMP mjd 53000 54200 0.0012 1
DMJUMP mjd 55500 56700 -0.0007
DMEFAC mjd 54000 56700 1.3
DMEQUAD mjd 53000 55000 0.0002
"""


def build():
    """(par text, model, TOAs) of wb_dd (seeded: the same TOAs on every call)."""
    np.random.seed(21)
    par = pta_par(21, "DD") + EXTRA
    model = get_model(io.StringIO(par))
    ts = sim.make_fake_toas_uniform(53000, 56652, 600, model, freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                    obs="geocenter", error=0.5 * u.us, add_noise=True, add_correlated_noise=True,
                                    include_bipm=False, multi_freqs_in_epoch=False, wideband=True,
                                    wideband_dm_error=2e-4 * u.pc / u.cm ** 3)
    model.find_empty_masks(ts, freeze=True)
    return par, model, ts


def main():
    register_clockless_sites()
    par, model, ts = build()
    with open(f"{GOLDEN}/wb_dd.par", "w") as f:
        f.write(par)
    arr, flags = pack_toas(ts)
    tz = model.get_TZR_toa(ts)
    tza, _ = pack_toas(tz)
    arrays = dict(arr)
    arrays.update({"tzr_" + k: v for k, v in tza.items()})
    arrays.update(mask_table(model, ts))
    arrays.update(component_delays(model, ts))
    arrays.update(phase_outputs(model, ts))
    r, ra, rm = residual_outputs(model, ts)
    arrays.update(ra)
    no, nm = noise_outputs(model, ts)
    arrays.update(no)
    dm, dme = ts.get_dms().to_value(u.pc / u.cm ** 3), ts.get_dm_errors().to_value(u.pc / u.cm ** 3)
    arrays["wb_pp_dm"] = np.asarray(dm, dtype=np.float64)
    arrays["wb_pp_dme"] = np.asarray(dme, dtype=np.float64)
    wr = WidebandDMResiduals(ts, model)
    arrays["wb_total_dm"] = np.asarray(model.total_dm(ts).to_value(u.pc / u.cm ** 3), dtype=np.float64)
    arrays["wb_dm_resids"] = np.asarray(wr.resids.to_value(u.pc / u.cm ** 3), dtype=np.float64)
    arrays["wb_dm_sigma"] = np.asarray(wr.get_data_error().to_value(u.pc / u.cm ** 3), dtype=np.float64)
    wm = WidebandDMResiduals(ts, model, subtract_mean=True)
    arrays["wb_dm_resids_mean"] = np.asarray(wm.resids.to_value(u.pc / u.cm ** 3), dtype=np.float64)
    meta = {"name": "wb_dd", "model": export_model(model), "flags": flags}
    meta.update(rm)
    meta.update(nm)
    meta["wb_dm_chi2"] = float(wr.chi2)
    meta["wb_dm_dof"] = int(wr.dof)
    meta["wb_dm_rms_weighted"] = float(wr.rms_weighted().to_value(u.pc / u.cm ** 3))
    wt = WidebandTOAResiduals(ts, model)
    meta["wb_chi2"] = float(wt.chi2)
    meta["wb_dof"] = int(wt.dof)
    meta["wb_reduced_chi2"] = float(wt.reduced_chi2)
    meta["wb_toa_chi2"] = float(wt.toa.chi2)
    meta["wb_dm_chi2_combined"] = float(wt.dm.chi2)
    rw = wt.rms_weighted()
    meta["wb_rms_weighted"] = {"toa_us": float(rw["toa"].to_value(u.us)),
                               "dm": float(rw["dm"].to_value(u.pc / u.cm ** 3))}
    # WidebandTOAFitter (fitter.py:2292-2637): one GLS step over [TOA rows; DM rows]
    f = WidebandTOAFitter(ts, copy.deepcopy(model))
    chi2 = f.fit_toas(maxiter=1)
    meta["wbfit_chi2"] = float(chi2)
    meta["wbfit_params"] = {p: list(map(float, split_ld(getattr(f.model, p).value))) for p in f.model.free_params}
    meta["wbfit_errors"] = {p: float(getattr(f.model, p).uncertainty_value) for p in f.model.free_params}
    meta["wbfit_post_chi2"] = float(f.resids.chi2)
    arrays["wbfit_post_toa_resid"] = np.asarray(f.resids.toa.time_resids.to_value(u.s), dtype=np.float64)
    arrays["wbfit_post_dm_resid"] = np.asarray(f.resids.dm.resids.to_value(u.pc / u.cm ** 3), dtype=np.float64)
    arrays["wbfit_cov"] = np.asarray(f.parameter_covariance_matrix.matrix, dtype=np.float64)
    # WidebandDownhillFitter (fitter.py:1812-1895): the downhill line search on the combined chi2
    fd = WidebandDownhillFitter(ts, copy.deepcopy(model))
    try:
        fd.fit_toas(maxiter=10)
        meta["wbdown_status"] = "converged"
    except Exception as e:
        meta["wbdown_status"] = type(e).__name__
    meta["wbdown_chi2"] = float(fd.resids.chi2)
    meta["wbdown_params"] = {p: list(map(float, split_ld(getattr(fd.model, p).value))) for p in fd.model.free_params}
    meta["wbdown_errors"] = {p: float(getattr(fd.model, p).uncertainty_value) for p in fd.model.free_params}
    save("wb_dd", arrays, meta)


if __name__ == "__main__":
    main()
