"""Container-only check of pint_amd.interop (TEST INFRASTRUCTURE; run by
tests/test_interop.py through oracle/refenv/run_ref.sh).

Loads NGC6440E and B1855+09 with the reference exactly as the fixture generators do,
converts them with pint_amd.interop.from_pint, and reports -- as one JSON line -- whether
the packed columns, the TZR TOA and every parameter value equal the committed fixtures
(which the reference produced), and the residuals the CPU oracle computes from the
converted objects against the reference's own residuals."""
import json
import os
import sys

import numpy as np

from refcommon import REPO, REFDATA, GOLDEN, register_clockless_sites
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pint.toa as toa
from pint.models import get_model

from pint_amd import interop
import pint_oracle as O


def check(name, par, tim):
    model = get_model(f"{REFDATA}/{par}")
    toas = toa.get_TOAs(f"{REFDATA}/{tim}", ephem="builtin", include_bipm=False, planets=False, model=model)
    pm, pt = interop.from_pint(model, toas)
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    out = {}
    cols = ["tdb_hi", "tdb_lo", "freq_mhz", "err_us", "ssb_obs_pos_km", "ssb_obs_vel_kms", "obs_sun_pos_km",
            "mjd_float", "delta_pulse_number"]
    # max relative difference per column: the reference's own posvel computation is not
    # bit-reproducible run to run (1-ulp differences on a few B1855 TOAs)
    out["columns_maxrel"] = {c: float(np.max(np.abs(pt.arrays[c] - z[c])) / max(np.max(np.abs(z[c])), 1e-300))
                             for c in cols}
    out["tzr_equal"] = {c: bool(np.array_equal(np.atleast_1d(pt.tzr[c]), z["tzr_" + c]))
                        for c in ("tdb_hi", "tdb_lo", "freq_mhz", "ssb_obs_pos_km")}
    bad = {}
    for p, d in meta["model"]["values"].items():
        v = d.get("value")
        if p not in pm or not isinstance(v, list):
            continue
        ours = pm[p].value
        if ours is None:
            bad[p] = "missing"
            continue
        ref = np.longdouble(v[0]) + np.longdouble(v[1])
        if np.longdouble(ours) != ref and abs(float(np.longdouble(ours) - ref)) > 1e-15 * max(1.0, abs(float(ref))):
            bad[p] = [float(np.longdouble(ours)), float(ref)]
    out["param_mismatch"] = bad
    out["free_params_equal"] = list(pm.free_params) == list(meta["model"]["free_params"])
    r = O.residuals(O.from_product_model(pm), O.toas_from_product(pt))
    out["resid_max_abs_s"] = float(np.max(np.abs(r["time"] - z["res_time"])))
    return out


if __name__ == "__main__":
    register_clockless_sites()
    res = {"ngc6440e": check("ngc6440e", "NGC6440E.par", "NGC6440E.tim"),
           "b1855": check("b1855", "B1855+09_NANOGrav_9yv1.gls.par", "B1855+09_NANOGrav_9yv1.tim")}
    print("INTEROP " + json.dumps(res))
