"""PLANET_SHAPIRO (solar_system_shapiro.py:105-124): the five planets' Shapiro delays from
obs_<planet>_pos (toa.py:2403-2433 compute_posvels(planets=True)), against the reference run
with PLANET_SHAPIRO Y (tests/golden/planet_*.npz by oracle/refgen/gen_planets.py).

CPU: the oracle's delays against the reference's, the host preparation's planet vectors
(builtin ephemeris: erfa.plan94 + epv00, tabulated in pint_amd/data/prep_tables.npz) against
the reference's columns.  GPU: delays, residuals and fits through the C-ABI."""
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN, load, ref_value

import pint_oracle as O

LD = np.longdouble
PLANETS = ("jupiter", "saturn", "venus", "uranus", "neptune", "earth")


def _b1855_ref():
    z = dict(np.load(os.path.join(GOLDEN, "planet_b1855.npz"), allow_pickle=False))
    meta = json.load(open(os.path.join(GOLDEN, "planet_b1855.json")))
    return z, meta


def _from_tim(name):
    from pint_amd.toa import get_model_and_toas
    tim = {"planet_ngc": "NGC6440E.tim", "planet_b1855": "B1855+09_NANOGrav_9yv1.tim.gz"}[name]
    return get_model_and_toas(os.path.join(GOLDEN, f"{name}.par"), os.path.join(GOLDEN, tim), ephem="builtin",
                              include_bipm=False)


def test_planet_fixture_has_effect():
    """The planets move the Shapiro delay by tens of ns here: well above the 1 ns bar."""
    p = np.load(os.path.join(GOLDEN, "planet_ngc.npz"))
    s = np.load(os.path.join(GOLDEN, "ngc6440e.npz"))
    d = np.abs(p["delay_solar_system_shapiro_delay"] - s["delay_solar_system_shapiro_delay"])
    assert d.max() > 1e-8


def test_oracle_planet_delays():
    model, toas, z, meta = load("planet_ngc")
    assert model.PLANET_SHAPIRO.value and toas.planets
    om = O.from_fixture(meta)
    ev = O.evaluate(om, O.toas_from_fixture(z, meta))
    n = toas.ntoas
    assert np.max(np.abs(ev["shapiro"][:n] - z["delay_solar_system_shapiro_delay"])) < 1e-13
    assert np.max(np.abs(ev["delay"][:n] - z["delay_total"])) < 5e-12
    assert abs(ev["delay"][n] - z["tzr_delay"][0]) < 5e-12


@pytest.mark.parametrize("name", ["planet_ngc", "planet_b1855"])
def test_prep_planet_vectors(name):
    """load_tim with the model's PLANET_SHAPIRO Y prepares obs_<planet>_pos for the TOAs and
    the TZR TOA; the vectors agree with the reference's to the ephemeris-table floor."""
    m, t = _from_tim(name)
    assert t.planets
    if name == "planet_ngc":
        z = np.load(os.path.join(GOLDEN, "planet_ngc.npz"))
        rows = np.arange(t.ntoas)
        tz = t.tzr_for(m)
        for pl in PLANETS:
            assert np.max(np.abs(tz[f"obs_{pl}_pos_km"] - z[f"tzr_obs_{pl}_pos_km"])) < 2e-3, pl
    else:
        z, _ = _b1855_ref()
        rows = z["rows"]
    for pl in PLANETS:
        d = np.max(np.abs(t.arrays[f"obs_{pl}_pos_km"][rows] - z[f"obs_{pl}_pos_km"]))
        # measured 0.4 m for the planets (7e-7 km for the Earth): the planet table's floor.
        # The Shapiro delay moves by 2 T_planet dr/(r - r cos) ~ 1e-20 s per metre
        assert d < 2e-3, (pl, d)


def test_planets_false_has_no_columns():
    from pint_amd.toa import load_tim
    t = load_tim(os.path.join(GOLDEN, "NGC6440E.tim"), ephem="builtin", include_bipm=False, planets=False)
    assert not t.planets


@pytest.mark.gpu
def test_planet_delays_residuals_fit_ngc():
    from pint_amd import Residuals, WLSFitter
    from pint_amd.engine import evaluate_delay_phase
    model, toas, z, meta = load("planet_ngc")
    dp = evaluate_delay_phase(model, toas)
    assert np.max(np.abs(dp["delay"] - z["delay_total"])) < 5e-12
    assert abs(dp["tzr_delay"] - z["tzr_delay"][0]) < 5e-12
    r = Residuals(toas, model)
    assert np.max(np.abs(r.time_resids - z["res_time"])) < 1e-10
    f = WLSFitter(toas, model)
    c2 = f.fit_toas(maxiter=1)
    assert abs(c2 / meta["wls_chi2"] - 1) < 1e-7
    for p in meta["wls_params"]:
        s = meta["wls_errors"][p]
        d = float((LD(f.model[p].value) - ref_value(meta, "wls_params", p)) / LD(s))
        assert abs(d) < 1e-3, (p, d)


@pytest.mark.gpu
def test_planet_b1855_from_tim():
    """B1855+09 with PLANET_SHAPIRO Y prepared from its tim file: residuals within 1 ns of the
    reference's and its GLS fit (bars of test_prep.py::test_residuals_and_fit_from_tim)."""
    from pint_amd import GLSFitter, Residuals
    m, t = _from_tim("planet_b1855")
    z, meta = _b1855_ref()
    m.free_params = [p for p in meta["model"]["free_params"] if p in m]
    r = Residuals(t, m)
    assert np.max(np.abs(r.time_resids - z["res_time"])) < 1e-9
    f = GLSFitter(t, m)
    chi2 = f.fit_toas(maxiter=1)
    assert abs(chi2 / meta["gls_chi2"] - 1) < 1e-5
    for p, (hi, lo) in meta["gls_params"].items():
        sig = meta["gls_errors"][p]
        assert abs(float(LD(f.model[p].value) - (LD(hi) + LD(lo)))) < 5e-3 * sig, p


@pytest.mark.gpu
def test_planet_shapiro_needs_planet_columns():
    """Like the reference (solar_system_shapiro.py:118-122): PLANET_SHAPIRO Y with TOAs loaded
    without planets is a KeyError naming planets=True."""
    from pint_amd import Residuals
    from pint_amd.toa import load_tim
    model, _, _, _ = load("planet_ngc")
    t = load_tim(os.path.join(GOLDEN, "NGC6440E.tim"), model=model, ephem="builtin", include_bipm=False,
                 planets=False)
    with pytest.raises(KeyError, match="planets=True"):
        Residuals(t, model)
