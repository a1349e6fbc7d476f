"""Time/ephemeris tables for host TOA preparation (container only).

The reference prepares TOAs with astropy/erfa (toa.py:2251 compute_TDBs, :2323
compute_posvels; observatory/topo_obs.py posvel; erfautils.py gcrs_posvel_from_itrf ->
EarthLocation.get_gcrs_posvel).  The GPU box has neither, so pint_amd/prep.py evaluates the
same quantities from these tables (data, sampled from the reference's own environment:
astropy 4.3.1, pyerfa 2.0.0, ephem="builtin", IERS-B bundled with astropy):

* leap seconds   : erfa.dat at every month start 1972-2030 -> (mjd, TAI-UTC) steps
* iers           : the IERS-B table astropy uses offline (MJD, PM_x, PM_y [arcsec],
                   UT1_UTC [s]) -- interpolated by pint_amd.prep exactly as astropy's
                   IERS._interpolate does (linear, leap-second-corrected UT1-UTC)
* cip            : erfa.xys06a (IAU 2006/2000A CIP X, Y and CIO locator s, rad) at TT,
                   0.5-day grid (cubic interpolation: < 1 uas)
* dtdb           : erfa.dtdb's decomposition dtdb = G(t) + u [sin(tsol) C(t) + cos(tsol) S(t)]
                   + v B(t) (tsol = 2 pi ut + elong; checked to 1e-14 s) at TT, 0.5-day grid
* earth          : erfa.epv00 barycentric Earth position (km) / velocity (km/s) at TDB,
                   0.25-day grid (6-point Lagrange: < 2 cm)
* sun            : Sun barycentric position/velocity (epv00 pvb - pvh), 1-day grid
* venus, jupiter, saturn, uranus, neptune
                 : barycentric positions (km) as astropy 4.3's builtin
                   get_body_barycentric_posvel forms them (erfa.plan94 heliocentric + the
                   Sun's epv00 barycentric vector) for compute_posvels(planets=True)
                   (toa.py:2403-2433); Venus on a 1-day grid, the outer planets on 4 days
                   (6-point Lagrange: < 10 m, checked below)
Usage: run_ref.sh gen_prep_tables.py
"""
import os
import sys

import numpy as np
import erfa
from astropy.utils import iers

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
AU_KM = 149597870.7
DAYSEC = 86400.0
M0, M1 = 49900.0, 60600.0


def planet_bary_km(mjd, idx):
    """astropy 4.3 _get_body_barycentric_posvel for ephemeris 'builtin': erfa.plan94
    heliocentric position plus the Sun's barycentric one (epv00 pvb - pvh), au -> km."""
    j1 = np.full_like(mjd, 2400000.5)
    pvh, pvb = erfa.epv00(j1, mjd)
    pl = erfa.plan94(j1, mjd, idx)
    return (pl["p"] + pvb["p"] - pvh["p"]) * AU_KM


def main():
    # leap seconds
    steps = []
    prev = None
    for y in range(1972, 2031):
        for m in range(1, 13):
            d = erfa.dat(y, m, 1, 0.0)
            if d != prev:
                jd1, jd2 = erfa.cal2jd(y, m, 1)
                steps.append((jd1 - 2400000.5 + jd2, d))
                prev = d
    leap = np.array(steps)
    # IERS-B as astropy uses it
    t = iers.earth_orientation_table.get()
    mjd = np.asarray(t["MJD"].value)
    sel = (mjd >= M0 - 2) & (mjd <= M1 + 2)
    iers_tab = np.column_stack([mjd[sel], np.asarray(t["PM_x"].to_value("arcsec"))[sel],
                                np.asarray(t["PM_y"].to_value("arcsec"))[sel],
                                np.asarray(t["UT1_UTC"].to_value("s"))[sel]])
    # CIP X, Y, s at TT
    g2 = np.arange(M0, M1 + 1e-9, 0.5)
    x, y, s = erfa.xys06a(np.full_like(g2, 2400000.5), g2)
    # dtdb decomposition at TT
    j1 = np.full_like(g2, 2400000.5)
    G = erfa.dtdb(j1, g2, 0.0, 0.0, 0.0, 0.0)
    S = erfa.dtdb(j1, g2, 0.0, 0.0, 1.0, 0.0) - G
    C = erfa.dtdb(j1, g2, 0.25, 0.0, 1.0, 0.0) - G
    B = erfa.dtdb(j1, g2, 0.0, 0.0, 0.0, 1.0) - G
    # check the decomposition at random arguments
    rng = np.random.default_rng(0)
    for _ in range(200):
        jd2 = rng.uniform(M0, M1)
        ut, el, u, v = rng.uniform(0, 1), rng.uniform(-np.pi, np.pi), rng.uniform(0, 6400), rng.uniform(-6400, 6400)
        full = erfa.dtdb(2400000.5, jd2, ut, el, u, v)
        g = erfa.dtdb(2400000.5, jd2, 0.0, 0.0, 0.0, 0.0)
        ss = erfa.dtdb(2400000.5, jd2, 0.0, 0.0, 1.0, 0.0) - g
        cc = erfa.dtdb(2400000.5, jd2, 0.25, 0.0, 1.0, 0.0) - g
        bb = erfa.dtdb(2400000.5, jd2, 0.0, 0.0, 0.0, 1.0) - g
        ts = (ut % 1.0) * 2 * np.pi + el
        assert abs(full - (g + u * (np.sin(ts) * cc + np.cos(ts) * ss) + v * bb)) < 1e-14, full
    # Earth at TDB
    g4 = np.arange(M0, M1 + 1e-9, 0.25)
    pvh, pvb = erfa.epv00(np.full_like(g4, 2400000.5), g4)
    earth = np.column_stack([pvb["p"] * AU_KM, pvb["v"] * AU_KM / DAYSEC])
    g1 = np.arange(M0, M1 + 1e-9, 1.0)
    pvh1, pvb1 = erfa.epv00(np.full_like(g1, 2400000.5), g1)
    sun = np.column_stack([(pvb1["p"] - pvh1["p"]) * AU_KM, (pvb1["v"] - pvh1["v"]) * AU_KM / DAYSEC])
    planets = {}
    for name, idx, step in (("venus", 2, 1.0), ("jupiter", 5, 4.0), ("saturn", 6, 4.0), ("uranus", 7, 4.0),
                            ("neptune", 8, 4.0)):
        gp = np.arange(M0, M1 + 1e-9, step)
        planets[name] = planet_bary_km(gp, idx)
        planets[name + "_t0"], planets[name + "_dt"] = M0, step
        # 6-point Lagrange (nodes i-2..i+3, as pint_amd.prep._lagrange6) at random epochs
        tt = rng.uniform(M0 + 3 * step, M1 - 4 * step, 300)
        xg = (tt - M0) / step
        i = np.floor(xg).astype(int)
        uu = xg - i
        est = 0.0
        for k in range(-2, 4):
            w = np.ones_like(uu)
            for m in range(-2, 4):
                if m != k:
                    w = w * (uu - m) / (k - m)
            est = est + w[:, None] * planets[name][i + k]
        err = np.max(np.abs(est - planet_bary_km(tt, idx)))
        assert err < 1e-2, (name, err)
    out = os.path.join(REPO, "pint_amd", "data", "prep_tables.npz")
    np.savez_compressed(out, leap=leap, iers=iers_tab, cip_t0=M0, cip_dt=0.5, cip=np.column_stack([x, y, s]),
                        dtdb_t0=M0, dtdb_dt=0.5, dtdb=np.column_stack([G, C, S, B]),
                        earth_t0=M0, earth_dt=0.25, earth=earth, sun_t0=M0, sun_dt=1.0, sun=sun, **planets,
                        source=np.array("astropy 4.3.1 / pyerfa 2.0.0 (ephem builtin, IERS-B), "
                                        "oracle/refgen/gen_prep_tables.py"))
    print("wrote", out, os.path.getsize(out), "iers", iers_tab[0, 0], iers_tab[-1, 0], file=sys.stderr)


if __name__ == "__main__":
    main()
