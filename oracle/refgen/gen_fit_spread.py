"""The reference's own chi2 spread per fixture (reference run; container only; TEST
INFRASTRUCTURE).  Writes tests/golden/fit_spread.json, from which the end-to-end chi2 bars of
the GPU tests are set (2x the spread) instead of one blanket relative bar.

Two correct evaluations of a timing model -- the reference's numpy longdouble and the
device's double-double -- give time residuals that differ by a few to a few tens of ps per TOA
(the residual tests hold the device to <= 30 ps rms of the reference's).  A chi2 computed from
such residuals moves with them, by an amount that depends on the fixture (TOA errors, count,
correlated noise).  This script measures that for the reference itself: every time residual
it computes (Residuals.calc_time_resids, residuals.py:483) is shifted by a fixed per-TOA
pattern of rms sigma_p (5 ps, the longdouble floor, and 30 ps, the residual tests' rms bar),
and the pre-fit Residuals chi2, the GLSFitter / WLSFitter fit_toas(maxiter=1) chi2 and (for
the Downhill fixtures) the DownhillGLSFitter chi2 are recorded as max |chi2 / chi2_0 - 1|.
The patterns are NREP independent N(0, sigma_p) draws and, because two evaluations' residual
differences are not independent per TOA (they follow the TOA epoch and frequency), four
structured ones of the same rms: sinusoids in time over the data span, a third of it and one
year (random phase), and a dispersive (1400 MHz / f)^2 pattern with zero weighted mean.

The (model, TOAs) of each fixture are rebuilt by its own generator (gen_synth, gen_phoff,
gen_stage.rebuild), whose capture() is intercepted, and checked bit-for-bit against the
committed fixture's packed tdb.

Usage: oracle/refenv/run_ref.sh oracle/refgen/gen_fit_spread.py [name ...]
"""
import copy
import json
import os
import sys

import numpy as np
import astropy.units as u

from refcommon import GOLDEN, register_clockless_sites
import pint.fitter as pfit
import pint.residuals as pres

import gen_phoff
import gen_synth

NREP = 4
LEVELS = {"5ps": 5e-12, "30ps": 3e-11}
DOWNHILL = {"pta_iso", "pta_ell1", "pta_dd", "ecorr_phoff", "phoff_red", "phoff_ecorr", "phoff_dmn", "j0740"}

_GRAB = {}


def _grab(name, model, toas, fit="gls", n_dm_rows=None):
    _GRAB[name] = (model, toas, fit)


gen_synth.capture = _grab
gen_phoff.capture = _grab

SYNTH = {"pta_iso": (1, ""), "pta_ell1": (2, "ELL1"), "pta_dd": (3, "DD"), "pta_bt": (14, "BT"),
         "pta_ddk": (16, "DDK"), "pta_ddk_nk": (17, "DDK_NK"), "ell1h_h3": (11, "ELL1H_H3"),
         "ell1h_h4": (12, "ELL1H_H4"), "ell1h_stig": (13, "ELL1H_STIG")}
PHOFF = {"wls_phoff": (5, False, "wls", False), "ecorr_phoff": (6, True, "gls", False),
         "phoff_red": (7, False, "gls", True), "phoff_ecorr": (8, True, "gls", True),
         "phoff_dmn": (9, False, "gls", True)}


def rebuild(name):
    _GRAB.clear()
    if name in SYNTH:
        gen_synth.gen_pta(*SYNTH[name])
    elif name == "pta_dmn":
        gen_synth.extra_name = "pta_dmn"
        gen_synth.gen_pta(15, "ELL1", extra="TNDMAMP -13.2\nTNDMGAM 2.8\nTNDMC 20\n")
        gen_synth.extra_name = None
    elif name == "j0740":
        gen_synth.gen_j0740()
    elif name in PHOFF:
        seed, ecorr, fit, frozen = PHOFF[name]
        gen_phoff.gen(name, seed, ecorr, fit, frozen=frozen, dmn=name == "phoff_dmn")
    elif name == "b1855":
        from gen_stage import rebuild as stage_rebuild
        m, t = stage_rebuild("b1855")
        return m, t, "gls"
    elif name == "ngc6440e":
        import pint.toa as toa
        from refcommon import REFDATA
        from pint.models import get_model
        m = get_model(f"{REFDATA}/NGC6440E.par")
        t = toa.get_TOAs(f"{REFDATA}/NGC6440E.tim", ephem="builtin", include_bipm=False, planets=False, model=m)
        return m, t, "wls"
    elif name == "wls_noise":
        import gen_noise
        par = gen_noise.par_white(7)
        m, t = gen_noise.toas_for(7, False, par)
        return m, t, "wls"
    elif name == "white_mjd":
        import io
        import gen_noise
        import pint.simulation as sim
        from pint.models import get_model
        np.random.seed(11)
        m = get_model(io.StringIO(gen_noise.WHITE_MJD_PAR))
        t = sim.make_fake_toas_uniform(50000, 55000, 200, m, add_noise=True, include_bipm=False)
        return gen_noise.frozen_noise(m), t, "wls"
    elif name == "ecorr_fit":
        import gen_noise
        import pint.toa as toa
        from refcommon import REFDATA
        from pint.models import get_model
        m = get_model(f"{REFDATA}/ecorr_fit_test.par")
        t = toa.get_TOAs(f"{REFDATA}/ecorr_fit_test.tim", ephem="builtin", include_bipm=False, planets=False, model=m)
        return gen_noise.frozen_noise(m), t, "gls"
    elif name == "wb_dd":
        import gen_wideband
        _, m, t = gen_wideband.build()
        return m, t, "wb"
    elif name in ("c5_iso", "c5_ell1", "c5_dd"):
        import io
        import pint.simulation as sim
        from pint.models import get_model
        seed, binary = {"c5_iso": (0, ""), "c5_ell1": (1, "ELL1"), "c5_dd": (2, "DD")}[name]
        np.random.seed(seed)
        m = get_model(io.StringIO(gen_synth.pta_par(seed, binary, ndmx=100)))
        t = sim.make_fake_toas_uniform(53000, 56652, 10000, m, freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                       obs="geocenter", error=0.5 * u.us, add_noise=True, add_correlated_noise=True,
                                       include_bipm=False, multi_freqs_in_epoch=False)
        m.find_empty_masks(t, freeze=True)
        return m, t, "gls"
    else:
        raise KeyError(name)
    m, t, fit = _GRAB[name]
    return m, t, fit


def check_same(name, toas):
    base = np.load(os.path.join(GOLDEN, name + ".npz"))
    assert np.array_equal(np.asarray(toas.table["tdbld"], dtype=np.float64), base["tdb_hi"]), f"{name}: TOAs differ"


def patterns(toas):
    """Unit-rms residual shift patterns: NREP N(0, 1) draws, then the structured ones."""
    out = [np.random.default_rng(rep).normal(0.0, 1.0, toas.ntoas) for rep in range(1, NREP + 1)]
    t = np.asarray(toas.table["tdbld"], dtype=np.float64)
    span = max(t.max() - t.min(), 1.0)
    rng = np.random.default_rng(100)
    for per in (span, span / 3.0, 365.25):
        p = np.sin(2 * np.pi * (t - t.min()) / per + rng.uniform(0, 2 * np.pi))
        out.append(p / np.sqrt(np.mean(p * p)))
    f = np.asarray(toas.get_freqs().to_value(u.MHz), dtype=np.float64)
    p = (1400.0 / np.where(np.isfinite(f) & (f > 0), f, 1400.0)) ** 2
    p = p - np.mean(p)
    out.append(p / np.sqrt(np.mean(p * p)) if np.any(p) else out[0])
    return out


def measure(model, toas, fit, down):
    fcls = pfit.GLSFitter if fit == "gls" else pfit.WLSFitter
    keys = ("pre", "fit", "down", "post")

    def run():
        if fit == "wb":  # wb_dd: WidebandTOAResiduals, WidebandTOAFitter (linearised and post-fit
            # chi2), WidebandDownhillFitter; the TOA part of the residuals carries the shift
            pre = float(pres.WidebandTOAResiduals(toas, model).chi2)
            f = pfit.WidebandTOAFitter(toas, copy.deepcopy(model))
            c = float(f.fit_toas(maxiter=1))
            post = float(f.resids.chi2)
            fd = pfit.WidebandDownhillFitter(toas, copy.deepcopy(model))
            try:
                fd.fit_toas(maxiter=10)
            except Exception:
                pass
            return pre, c, float(fd.resids.chi2), post
        pre = float(pres.Residuals(toas, model).chi2)
        f = fcls(toas, copy.deepcopy(model))
        c = float(f.fit_toas(maxiter=1))
        d = None
        if down:
            fd = pfit.DownhillGLSFitter(toas, copy.deepcopy(model))
            try:
                fd.fit_toas(maxiter=10)
            except Exception:
                pass
            d = float(fd.resids.chi2)
        return pre, c, d, None

    base = run()
    out = {"chi2_0": dict(zip(keys, base)), "nrep": NREP}
    orig = pres.Residuals.calc_time_resids
    try:
        for key, sig in LEVELS.items():
            worst = {k: (0.0 if v is not None else None) for k, v in zip(keys, base)}
            for rep, pat in enumerate(patterns(toas), start=1):
                shift = pat * sig * u.s

                def calc(self, *a, **k):
                    return orig(self, *a, **k) + shift
                pres.Residuals.calc_time_resids = calc
                got = run()
                pres.Residuals.calc_time_resids = orig
                for j, k in enumerate(keys):
                    if got[j] is not None:
                        worst[k] = max(worst[k], abs(got[j] / base[j] - 1))
            out[key] = worst
    finally:
        pres.Residuals.calc_time_resids = orig
    return out


if __name__ == "__main__":
    register_clockless_sites()
    path = os.path.join(GOLDEN, "fit_spread.json")
    res = json.load(open(path)) if os.path.exists(path) else {}
    names = sys.argv[1:] or (list(SYNTH) + ["pta_dmn", "j0740", "b1855"] + list(PHOFF) +
                             ["ngc6440e", "wls_noise", "white_mjd", "ecorr_fit", "c5_iso", "c5_ell1", "c5_dd"])
    for n in names:
        m, t, fit = rebuild(n)
        check_same(n, t)
        res[n] = measure(m, t, fit, n in DOWNHILL or fit == "wb")
        print(n, json.dumps(res[n]), file=sys.stderr, flush=True)
        with open(path, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
