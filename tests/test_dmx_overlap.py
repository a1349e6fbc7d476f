"""Overlapping DMX bins (dispersion_model.py:659-708): a TOA in any number of bins gets every
bin's DMX_ and a 1 in every bin's column.  The first two bins of a TOA travel as
pint_toas_t.dmx_a / dmx_b, the rest in the dmx_x CSR overflow.  Reference fixture:
NGC6440E with six free bins, TOAs in 3 and 4 bins (oracle/refgen/gen_dmx_overlap.py)."""
import numpy as np
import pytest

from golden_util import load, ref_value

import pint_oracle as O

LD = np.longdouble


def _bins_per_toa(model, toas):
    mjd = toas.get_mjds()
    cnt = np.zeros(toas.ntoas, dtype=int)
    for name in model.dmx_params():
        tag = name.split("_")[1]
        r1, r2 = float(model["DMXR1_" + tag].value), float(model["DMXR2_" + tag].value)
        cnt += (mjd >= r1) & (mjd <= r2)
    return cnt


def test_fixture_has_deep_overlap():
    model, toas, z, meta = load("dmx_overlap")
    cnt = _bins_per_toa(model, toas)
    assert cnt.max() == 4 and (cnt == 3).sum() >= 2 and (cnt == 0).sum() >= 6


def test_oracle_overlap_delays_and_columns():
    model, toas, z, meta = load("dmx_overlap")
    om = O.from_fixture(meta)
    T = O.toas_from_fixture(z, meta)
    ev = O.evaluate(om, T)
    n = toas.ntoas
    assert np.max(np.abs(ev["delay"][:n] - z["delay_total"])) < 5e-12
    M, names = O.designmatrix(om, T)
    ref = z["dm_M"][:, [list(meta["dm_params"]).index(p) for p in names]]
    scale = np.max(np.abs(ref), axis=0)
    scale[scale == 0] = 1
    assert np.max(np.abs(M - ref) / scale) < 1e-9


def test_pack_overflow_csr():
    """pack_toas: bins three and up in the dmx_x CSR (n+2 offsets, then indices), in
    parameter order; dmx_a/dmx_b hold the first two."""
    from pint_amd.engine import build_layout, pack_toas
    model, toas, z, meta = load("dmx_overlap")
    lay = build_layout(model, toas)
    t, keep = pack_toas(lay)
    da, db, x = keep[11], keep[12], keep[14]
    n = toas.ntoas
    assert x is not None and x[0] == n + 2 and x[n + 1] == len(x)
    mjd = np.concatenate([toas.get_mjds(), np.atleast_1d(toas.tzr["mjd_float"])])  # the TZR TOA too
    names = model.dmx_params()
    for i in range(n + 1):
        want = [j for j, nm in enumerate(names)
                if float(model["DMXR1_" + nm[4:]].value) <= mjd[i] <= float(model["DMXR2_" + nm[4:]].value)]
        got = [b for b in (da[i], db[i]) if b >= 0] + list(x[x[i]:x[i + 1]])
        assert got == want, (i, got, want)


@pytest.mark.gpu
def test_overlap_device_parity():
    from pint_amd import Residuals, WLSFitter
    from pint_amd.engine import evaluate_delay_phase
    model, toas, z, meta = load("dmx_overlap")
    dp = evaluate_delay_phase(model, toas)
    assert np.max(np.abs(dp["delay"] - z["delay_total"])) < 5e-12
    r = Residuals(toas, model)
    assert np.max(np.abs(r.time_resids - z["res_time"])) < 1e-10
    M, params, _ = model.designmatrix(toas)
    ref = z["dm_M"][:, [list(meta["dm_params"]).index(p) for p in params]]
    scale = np.max(np.abs(ref), axis=0)
    scale[scale == 0] = 1
    assert np.max(np.abs(M - ref) / scale) < 1e-9
    f = WLSFitter(toas, model)
    c2 = f.fit_toas(maxiter=1)
    assert abs(c2 / meta["wls_chi2"] - 1) < 1e-7
    for p in meta["wls_params"]:
        s = meta["wls_errors"][p]
        d = float((LD(f.model[p].value) - ref_value(meta, "wls_params", p)) / LD(s))
        assert abs(d) < 1e-3, (p, d)
        assert abs(f.model[p].uncertainty / s - 1) < 1e-6, p
