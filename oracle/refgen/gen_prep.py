"""Host TOA-preparation fixtures (reference run, container only).

The reference's get_TOAs (toa.py:109-330: read_toa_file :700, apply_clock_corrections
:2184, compute_TDBs :2251, compute_posvels :2323, phase_columns_from_flags :1959) on:
* NGC6440E.tim (Princeton format, GBT) with its model's TZR TOA;
* B1855+09_NANOGrav_9yv1.tim (Tempo2 format, Arecibo, -to TIME flags) with its TZR TOA;
* prep_mixed.tim, written here: Tempo2 + Princeton + an INCLUDEd Parkes-format file, sites
  gbt / arecibo / geocenter / barycenter, and the TIME, EFAC, EQUAD, EMIN, FMIN, JUMP,
  SKIP/NOSKIP, PHASE, INFO, MODE commands, -pn / -padd flags.
Offline recipe: ephem builtin, include_bipm False, planets False, clockless sites.
Also the clock file tests/datafile/wsrt2gps.clk read and evaluated (prep_clock.json).
Stage arrays: UTC / TT / TDB (jd1, jd2), the site's GCRS position/velocity, the Earth's
SSB position/velocity.  Writes tests/golden/prep_<name>.npz + .json.gz and the tim files.
"""
import gzip
import json
import os
import shutil
import sys

import numpy as np
import astropy.units as u

from refcommon import GOLDEN, REFDATA, register_clockless_sites, split_ld
import pint.toa as toa
from pint.models import get_model
from pint.observatory import get_observatory
from pint.solar_system_ephemerides import objPosVel_wrt_SSB
from pint.pulsar_mjd import Time

MIXED = """FORMAT 1
MODE 1
C a comment line
# another comment
mixed1 1400.0 55000.1234567890123456 1.0 gbt -f L-wide -be GUPPI
mixed2 820.0 55000.2234567890123 2.5 ao -f 430 -pn 100
TIME 0.5
mixed3 1400.0 55010.5 1.0 gbt -f L-wide
EFAC 2
EQUAD 1.5
mixed4 2000.0 55100.75 3.0 coe -f X
TIME -0.5
EFAC 1
EQUAD 0
JUMP
mixed5 1400.0 55200.3333333333333333 1.0 @ -f bary
JUMP
SKIP
skipped 1400.0 55300.1 1.0 gbt
NOSKIP
EMIN 0.5
mixed6 1400.0 55400.1 0.4 gbt
mixed6b 1400.0 55400.2 0.6 gbt
FMIN 900
mixed7 800.0 55500.1 1.0 gbt
mixed7b 1000.0 55500.2 1.0 gbt
PHASE 0.25
mixed8 1400.0 55600.123 1.0 gbt -padd 0.1
INFO myinfo
mixed9 0.0 55700.9 1.0 ao
INCLUDE prep_mixed_inc.tim
mixed10 1400.0 58000.000000000001 1.0 gbt
"""


def parkes_line(name, freq, imjd, frac13, err, obs):
    s = " " + name.ljust(24) + f"{freq:9.3f}" + f"{imjd:7d}" + "." + frac13 + f"{0.0:7.4f}" + " " + \
        f"{err:8.3f}" + " " * 8 + obs
    assert s[41] == "." and len(s) == 80
    return s


INC = "\n".join([
    parkes_line("pks1", 1369.0, 55800, "1234567890123", 2.0, "1"),
    "3              430.0000 55900.12345678901234    1.50",
    "1               1400.000 55950.5000000000000    0.80",
]) + "\n"


def stage_arrays(t):
    tab = t.table
    mjd = tab["mjd"]
    out = {}
    out["utc_jd1"] = np.array([m.jd1 for m in mjd], dtype=np.float64)
    out["utc_jd2"] = np.array([m.jd2 for m in mjd], dtype=np.float64)
    tdb = tab["tdb"]
    out["tdb_jd1"] = np.array([m.jd1 for m in tdb], dtype=np.float64)
    out["tdb_jd2"] = np.array([m.jd2 for m in tdb], dtype=np.float64)
    tt = np.array([m.tt for m in mjd])
    out["tt_jd1"] = np.array([x.jd1 for x in tt], dtype=np.float64)
    out["tt_jd2"] = np.array([x.jd2 for x in tt], dtype=np.float64)
    hi, lo = split_ld(tab["tdbld"])
    out["tdb_hi"], out["tdb_lo"] = hi, lo
    out["mjd_float"] = np.asarray(tab["mjd_float"], dtype=np.float64)
    out["err_us"] = np.asarray(tab["error"].quantity.to_value(u.us), dtype=np.float64)
    out["freq_mhz"] = np.asarray(tab["freq"].quantity.to_value(u.MHz), dtype=np.float64)
    out["ssb_obs_pos_km"] = np.asarray(tab["ssb_obs_pos"].quantity.to_value(u.km), dtype=np.float64)
    out["ssb_obs_vel_kms"] = np.asarray(tab["ssb_obs_vel"].quantity.to_value(u.km / u.s), dtype=np.float64)
    out["obs_sun_pos_km"] = np.asarray(tab["obs_sun_pos"].quantity.to_value(u.km), dtype=np.float64)
    out["delta_pulse_number"] = np.asarray(tab["delta_pulse_number"], dtype=np.float64)
    if "pulse_number" in tab.colnames:
        out["pulse_number"] = np.asarray(tab["pulse_number"], dtype=np.float64)
    ep = np.zeros((len(tab), 3))
    ev = np.zeros((len(tab), 3))
    for obs, grp in t.get_obs_groups():
        site = get_observatory(obs)
        tdbt = Time(tab[grp]["tdb"], precision=9)
        e = objPosVel_wrt_SSB("earth", tdbt, "builtin")
        ep[grp] = e.pos.T.to_value(u.km)
        ev[grp] = e.vel.T.to_value(u.km / u.s)
    # the site's GCRS vector is what compute_posvels added to the Earth's (topo_obs.py posvel)
    gp = out["ssb_obs_pos_km"] - ep
    gv = out["ssb_obs_vel_kms"] - ev
    out["gcrs_pos_km"], out["gcrs_vel_kms"] = gp, gv
    out["earth_pos_km"], out["earth_vel_kms"] = ep, ev
    meta = {"obs": [str(o) for o in tab["obs"]], "flags": [dict(f) for f in tab["flags"]],
            "commands": [[list(c[0]), int(c[1])] for c in getattr(t, "commands", [])]}
    return out, meta


def run(name, timfile, model=None):
    t = toa.get_TOAs(timfile, ephem="builtin", include_bipm=False, planets=False, model=model)
    arrays, meta = stage_arrays(t)
    if model is not None:
        tz = model.get_TZR_toa(t)
        ta, tm = stage_arrays(tz)
        arrays.update({"tzr_" + k: v for k, v in ta.items()})
        meta["tzr"] = tm
    np.savez_compressed(os.path.join(GOLDEN, f"prep_{name}.npz"), **arrays)
    with gzip.open(os.path.join(GOLDEN, f"prep_{name}.json.gz"), "wt") as f:
        json.dump(meta, f, default=str)
    print(name, len(t), file=sys.stderr)


def main():
    register_clockless_sites()
    dst = os.path.join(GOLDEN, "NGC6440E.tim")
    if os.path.exists(dst):
        os.chmod(dst, 0o644)
    shutil.copyfile(f"{REFDATA}/NGC6440E.tim", dst)
    os.chmod(dst, 0o644)
    with open(f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", "rb") as fi, \
            gzip.open(os.path.join(GOLDEN, "B1855+09_NANOGrav_9yv1.tim.gz"), "wb") as fo:
        fo.write(fi.read())
    with open(os.path.join(GOLDEN, "prep_mixed.tim"), "w") as f:
        f.write(MIXED)
    with open(os.path.join(GOLDEN, "prep_mixed_inc.tim"), "w") as f:
        f.write(INC)
    run("ngc6440e", f"{REFDATA}/NGC6440E.tim", get_model(f"{REFDATA}/NGC6440E.par"))
    run("b1855", f"{REFDATA}/B1855+09_NANOGrav_9yv1.tim", get_model(f"{REFDATA}/B1855+09_NANOGrav_9yv1.gls.par"))
    run("mixed", os.path.join(GOLDEN, "prep_mixed.tim"))
    # clock-file reading and interpolation (clock_file.py:432-546, :143-188)
    from pint.observatory.clock_file import read_tempo2_clock_file
    import warnings
    shutil.copyfile(f"{REFDATA}/wsrt2gps.clk", os.path.join(GOLDEN, "wsrt2gps.clk"))
    cf = read_tempo2_clock_file(f"{REFDATA}/wsrt2gps.clk")
    mjds = np.concatenate([[51000.0, 51179.5, 51179.75], np.linspace(51180.1, cf.time.mjd[-1] - 0.3, 37),
                           [cf.time.mjd[-1], cf.time.mjd[-1] + 10.0]])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        vals = cf.evaluate(Time(mjds, format="mjd", scale="utc")).to_value(u.s)
    with open(os.path.join(GOLDEN, "prep_clock.json"), "w") as f:
        json.dump({"file": "wsrt2gps.clk", "mjd": mjds.tolist(), "corr_s": np.asarray(vals).tolist(),
                   "n": int(len(cf.time)), "first": float(cf.time.mjd[0]), "last": float(cf.time.mjd[-1])}, f)


if __name__ == "__main__":
    main()
