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


@pytest.mark.parametrize("case", ["touching", "disjoint", "shuffled", "gaps_and_pairs", "nested"])
def test_pack_bin_assignment_matches_the_per_bin_rule(case):
    """pack_toas assigns bins by two sorted searches when the ranges are sorted with
    non-decreasing ends and no TOA lies in more than two bins (the PTA's consecutive bins
    share their endpoints); anything else takes the per-bin pass.  Both must give every TOA
    its selecting bins in parameter order (toa_select.py:101, inclusive)."""
    from pint_amd.engine import build_layout, pack_toas
    model, toas, z, meta = load("dmx_overlap")
    names = model.dmx_params()
    mjd = np.concatenate([toas.get_mjds(), np.atleast_1d(toas.tzr["mjd_float"])])
    rng = np.random.default_rng(7)
    lo, hi = float(mjd[:-1].min()), float(mjd[:-1].max())
    m = len(names)
    edges = np.linspace(lo - 1, hi + 1, m + 1)
    r1, r2 = edges[:-1].copy(), edges[1:].copy()
    if case == "touching":     # a TOA exactly on a shared endpoint is in both bins
        k = np.arange(1, m)   # each inner edge moved onto the nearest TOA
        r2[k - 1] = r1[k] = np.sort(mjd[np.argmin(np.abs(mjd[:-1, None] - edges[None, k]), axis=0)])
    elif case == "disjoint":
        r2 -= 1e-3
    elif case == "shuffled":   # parameter order != time order
        p = rng.permutation(m)
        r1, r2 = r1[p], r2[p]
    elif case == "gaps_and_pairs":
        r1[::2] += 0.3 * (r2[::2] - r1[::2])
        r2[1::2] = r2[1::2] + 0.5 * (edges[1] - edges[0])  # overlaps the next bin: pairs of bins
    else:                      # one bin inside another: the per-bin pass
        r1[1], r2[1] = r1[0] + 0.1, r2[0] - 0.1
    for nm, a, b in zip(names, r1, r2):
        model["DMXR1_" + nm[4:]].value = LD(a)
        model["DMXR2_" + nm[4:]].value = LD(b)
    t, keep = pack_toas(build_layout(model, toas))
    da, db, x = keep[11], keep[12], keep[14]
    if case == "touching":
        assert (db >= 0).sum() >= 1  # some TOA sits on a shared endpoint
    for i in range(len(mjd)):
        want = [j for j, nm in enumerate(names)
                if float(model["DMXR1_" + nm[4:]].value) <= mjd[i] <= float(model["DMXR2_" + nm[4:]].value)]
        got = [b for b in (da[i], db[i]) if b >= 0] + (list(x[x[i]:x[i + 1]]) if x is not None else [])
        assert got == want, (case, i, got, want)
