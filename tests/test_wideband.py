"""Wideband DM residuals (residuals.py:908-1271): the CPU oracle pinned to the reference's
fixture (wb_dd: DD + red noise, DMX, DMJUMP, DMEFAC, DMEQUAD on MJD ranges, make_fake_toas
wideband DMs; oracle/refgen/gen_wideband.py), and the HIP path (k_dm_resid through the
C-ABI) against both."""
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN, chi2_bar, rms_ps

import pint_oracle as O

LD = np.longdouble


def _fixture():
    z = dict(np.load(os.path.join(GOLDEN, "wb_dd.npz"), allow_pickle=False))
    meta = json.load(open(os.path.join(GOLDEN, "wb_dd.json")))
    return O.from_fixture(meta), O.toas_from_fixture(z, meta), z, meta


def test_oracle_total_dm_and_resids():
    om, toas, z, meta = _fixture()
    assert np.max(np.abs(O.total_dm(om, toas) - z["wb_total_dm"])) < 1e-12
    d = O.dm_residuals(om, toas)
    assert np.max(np.abs(d["resids"] - z["wb_dm_resids"])) < 1e-12
    assert np.max(np.abs(d["sigma"] / z["wb_dm_sigma"] - 1)) < 1e-15
    assert abs(d["chi2"] / meta["wb_dm_chi2"] - 1) < 1e-12
    dm = O.dm_residuals(om, toas, subtract_mean=True)
    assert np.max(np.abs(dm["resids"] - z["wb_dm_resids_mean"])) < 1e-12


def test_oracle_wideband_chi2():
    """The combined chi2 of the reference's WidebandTOAFitter pass = the TOA residuals' GLS
    chi2 + the DM chi2 (the TOA part at the end-to-end residual floor: 2x the reference's own
    chi2 spread at the measured residual rms, golden_util.chi2_bar)."""
    om, toas, z, meta = _fixture()
    c2 = O.wideband_chi2(om, toas)
    assert abs(c2 / meta["wb_chi2"] - 1) < chi2_bar("wb_dd", "pre", rms_ps(O.residuals(om, toas)["time"], z["res_time"]))
    assert abs(meta["wb_toa_chi2"] + meta["wb_dm_chi2_combined"] - meta["wb_chi2"]) < 1e-9 * meta["wb_chi2"]


@pytest.mark.gpu
def test_gpu_wideband_dm_resids():
    """WidebandDMResiduals on the GPU (k_dm_resid) against the reference's resids, scaled
    errors, chi2, dof and weighted RMS; with subtract_mean against the reference's too."""
    from golden_util import load
    from pint_amd import WidebandDMResiduals, Residuals
    model, toas, z, meta = load("wb_dd")
    r = Residuals(toas, model, residual_type="dm")
    assert isinstance(r, WidebandDMResiduals)
    assert np.max(np.abs(r.resids - z["wb_dm_resids"])) < 1e-12
    assert np.max(np.abs(r.get_data_error() / z["wb_dm_sigma"] - 1)) < 1e-15
    assert abs(r.chi2 / meta["wb_dm_chi2"] - 1) < 1e-12
    assert r.dof == meta["wb_dm_dof"]
    assert abs(r.rms_weighted() / meta["wb_dm_rms_weighted"] - 1) < 1e-10
    rm = WidebandDMResiduals(toas, model, subtract_mean=True)
    assert np.max(np.abs(rm.resids - z["wb_dm_resids_mean"])) < 1e-12


@pytest.mark.gpu
def test_gpu_wideband_toa_resids():
    """WidebandTOAResiduals: the reference's combined chi2 (its WidebandTOAFitter pass), dof,
    reduced chi2 and per-type weighted RMS; and the device's against the oracle's."""
    from golden_util import load
    from pint_amd import WidebandTOAResiduals
    model, toas, z, meta = load("wb_dd")
    w = WidebandTOAResiduals(toas, model)
    bar = chi2_bar("wb_dd", "pre", rms_ps(w.toa.time_resids, z["res_time"]))  # the TOA part's residual floor
    assert abs(w.chi2 / meta["wb_chi2"] - 1) < bar
    assert abs(w.dm.chi2 / meta["wb_dm_chi2_combined"] - 1) < 1e-12
    assert w.dof == meta["wb_dof"]
    assert abs(w.reduced_chi2 / meta["wb_reduced_chi2"] - 1) < bar
    rw = w.rms_weighted()
    assert abs(rw["toa"] / meta["wb_rms_weighted"]["toa_us"] - 1) < 1e-6
    assert abs(rw["dm"] / meta["wb_rms_weighted"]["dm"] - 1) < 1e-10
    om, ot, _, _ = _fixture()
    assert abs(w.dm.chi2 / O.dm_residuals(om, ot)["chi2"] - 1) < 1e-12
    # the TOA part: two independent dd / longdouble phase evaluations (~ps)
    ro = O.residuals(om, ot)["time"]
    assert abs(w.chi2 / O.wideband_chi2(om, ot) - 1) < chi2_bar("wb_dd", "pre", rms_ps(w.toa.time_resids, ro))
    with pytest.raises(AttributeError):
        w.dm.dof


def _ref_pars(meta, key):
    return {p: np.longdouble(v[0]) + np.longdouble(v[1]) for p, v in meta[key].items()}


def test_oracle_wideband_fit():
    """The oracle's WidebandTOAFitter step (fitter.py:2465-2637) against the reference's fit:
    parameters <= 1e-3 sigma (the TOA-residual floor), errors 1e-6, the linearised chi2 at
    the end-to-end floor."""
    om, toas, z, meta = _fixture()
    st = O.wideband_gls_step(om, toas)
    ref = _ref_pars(meta, "wbfit_params")
    for j, p in enumerate(st["names"]):
        if p == "Offset":
            continue
        sig = meta["wbfit_errors"][p]
        d = float(LD(om.values[p]) + LD(st["dpars"][j]) - ref[p]) / sig
        assert abs(d) < 1e-3, (p, d)
        assert abs(st["errs"][j] / sig - 1) < 1e-6, (p, st["errs"][j] / sig - 1)
    bar = chi2_bar("wb_dd", "fit", rms_ps(O.residuals(om, toas)["time"], z["res_time"]))
    assert abs(st["chi2"] / meta["wbfit_chi2"] - 1) < bar


@pytest.mark.gpu
def test_gpu_wideband_fit():
    """WidebandTOAFitter on the device (the DM rows added to the normal equations by
    k_wb_gram) against the reference's fit: parameters <= 1e-3 sigma, errors 1e-5, the
    linearised chi2 at the end-to-end floor; post-fit residuals; the model's DMDATA/DMRES."""
    from golden_util import load
    from pint_amd import WidebandTOAFitter
    model, toas, z, meta = load("wb_dd")
    f = WidebandTOAFitter(toas, model)
    c2 = f.fit_toas(maxiter=1)
    ref = _ref_pars(meta, "wbfit_params")
    worst = 0.0
    for p in meta["wbfit_params"]:
        s = meta["wbfit_errors"][p]
        d = float((LD(f.model[p].value) - ref[p]) / LD(s))
        worst = max(worst, abs(d))
        assert abs(f.model[p].uncertainty / s - 1) < 1e-5, (p, f.model[p].uncertainty / s - 1)
    assert worst < 1e-3, worst
    rms = rms_ps(f.resids.toa.time_resids, z["wbfit_post_toa_resid"])
    assert abs(c2 / meta["wbfit_chi2"] - 1) < chi2_bar("wb_dd", "fit", rms)
    assert abs(f.resids.chi2 / meta["wbfit_post_chi2"] - 1) < chi2_bar("wb_dd", "post", rms)
    assert np.max(np.abs(f.resids.toa.time_resids - z["wbfit_post_toa_resid"])) < 2e-10
    assert np.max(np.abs(f.resids.dm.resids - z["wbfit_post_dm_resid"])) < 1e-9
    assert f.model["DMDATA"].value is True and f.model["DMRES"].value > 0


@pytest.mark.gpu
def test_gpu_wideband_downhill():
    """WidebandDownhillFitter on the device (the wideband GLS step + the combined chi2 in the
    line search) against the reference's: status, chi2 at the end-to-end floor, and per
    parameter 2e-4 sigma or 2x the reference's own spread when its TOA residuals are perturbed
    at the 5 ps floor, where that is larger (downhill_spread.json["wb_dd"]: the nearly
    degenerate M2 / SINI pair and the orbital parameters move the reference's accepted iterate
    by up to 1.2e-3 sigma; the device measured 1.16e-3 sigma, SINI)."""
    from golden_util import load, downhill_bar
    from pint_amd import WidebandDownhillFitter
    from pint_amd.fitter import MaxiterReached, StepProblem
    model, toas, z, meta = load("wb_dd")
    f = WidebandDownhillFitter(toas, model)
    try:
        f.fit_toas(maxiter=10)
        status = "converged"
    except (MaxiterReached, StepProblem) as e:
        status = type(e).__name__
    assert status == meta["wbdown_status"]
    from pint_amd import Residuals
    bar = chi2_bar("wb_dd", "down", rms_ps(Residuals(toas, model).time_resids, z["res_time"]))
    assert abs(f.resids.chi2 / meta["wbdown_chi2"] - 1) < bar, (f.resids.chi2, meta["wbdown_chi2"], bar)
    ref = _ref_pars(meta, "wbdown_params")
    dev = {p: abs(float((LD(f.model[p].value) - ref[p]) / LD(meta["wbdown_errors"][p]))) for p in ref}
    p_w = max(dev, key=dev.get)
    print(f"wideband downhill: chi2 {f.resids.chi2:.6f} ref {meta['wbdown_chi2']:.6f}, worst {dev[p_w]:.2e} sigma ({p_w})")
    for p, d in dev.items():
        assert d < downhill_bar("wb_dd", p, floor=2e-4), (p, d, downhill_bar("wb_dd", p, floor=2e-4))


@pytest.mark.gpu
def test_gpu_wideband_fit_too_many_dm_columns():
    """k_wb_gram carries at most 8 free DM-type columns (DM Taylor terms + DMJUMPs); a model
    with more is refused (PINT_E_INVALID) instead of fitting the extra columns without their
    DM rows."""
    from golden_util import load
    from pint_amd import WidebandTOAFitter, get_model
    from pint_amd._lib import PintError
    model, toas, z, meta = load("wb_dd")
    text = open(os.path.join(GOLDEN, "wb_dd.par")).read()
    # 7 more free DMJUMPs on MJD ranges holding TOAs: DM, DM1, DM2 + 8 DMJUMPs = 11 columns
    extra = "".join(f"DMJUMP mjd {53000 + 400 * k} {53300 + 400 * k} 0.0 1\n" for k in range(1, 8))
    m2 = get_model(text + extra)
    m2.free_params = list(model.free_params) + [p for p in m2.params if p.startswith("DMJUMP")
                                                and p not in model.free_params]
    with pytest.raises((PintError, ValueError), match="DM-type columns"):
        WidebandTOAFitter(toas, m2).fit_toas(maxiter=1)
