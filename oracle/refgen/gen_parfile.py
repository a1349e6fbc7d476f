"""Reference as_parfile text (timing_model.py:2747, include_info=False) of the fixture models,
as read from their par files and after one GLS/WLS fit on the fixture TOAs (reference run,
container only).  Writes tests/golden/parfile_<name>.txt and parfile_<name>_fit.txt.
Usage: run_ref.sh gen_parfile.py [name ...]"""
import copy
import io
import json
import os
import sys

import numpy as np

from refcommon import GOLDEN, register_clockless_sites
from pint.models import get_model
from pint.fitter import GLSFitter, WLSFitter

PARS = {"ngc6440e": "NGC6440E.par", "b1855": "B1855+09_NANOGrav_9yv1.gls.par", "j0740": "J0740+6620.par",
        "pta_iso": "pta_iso.par", "pta_ell1": "pta_ell1.par", "pta_dd": "pta_dd.par",
        "wls_phoff": "wls_phoff.par", "ecorr_phoff": "ecorr_phoff.par", "wls_noise": "wls_noise.par",
        "ecorr_fit": "ecorr_fit.par", "white_mjd": "white_mjd.par",
        "ell1h_h3": "ell1h_h3.par", "ell1h_h4": "ell1h_h4.par", "ell1h_stig": "ell1h_stig.par",
        "pta_bt": "pta_bt.par", "pta_dmn": "pta_dmn.par", "pta_ddk": "pta_ddk.par", "pta_ddk_nk": "pta_ddk_nk.par", "wb_dd": "wb_dd.par",
        "c5_iso": "c5_iso.par", "c5_ell1": "c5_ell1.par", "c5_dd": "c5_dd.par",
        "planet_ngc": "planet_ngc.par", "planet_b1855": "planet_b1855.par",
        "dmx_overlap": "dmx_overlap.par", "phoff_red": "phoff_red.par", "phoff_ecorr": "phoff_ecorr.par",
        "phoff_dmn": "phoff_dmn.par"}




def main(names):
    register_clockless_sites()
    for name in names:
        m = get_model(os.path.join(GOLDEN, PARS[name]))
        with open(os.path.join(GOLDEN, f"parfile_{name}.txt"), "w") as f:
            f.write(m.as_parfile(include_info=False))
        if name in ("pta_dd", "j0740"):
            # the fixture's own GLS fit result (gls_params / gls_errors) written into the
            # model: the writer's formatting of fitted (longdouble-arithmetic) values, free of
            # the run-to-run BLAS noise a second fit would add
            meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
            mf = copy.deepcopy(m)
            for p in mf.params:
                getattr(mf, p).frozen = p not in meta["model"]["free_params"]
            for p, (hi, lo) in meta["gls_params"].items():
                par = getattr(mf, p)
                v = np.longdouble(hi) + np.longdouble(lo)
                par.value = v if isinstance(par.value, np.longdouble) or getattr(par, "long_double", False) or \
                    type(par).__name__ == "MJDParameter" else float(v)
                if type(par).__name__ == "AngleParameter":
                    par.uncertainty = meta["gls_errors"][p] * par.units  # (the value is in .units)
                else:
                    par.uncertainty_value = meta["gls_errors"][p]
            with open(os.path.join(GOLDEN, f"parfile_{name}_fit.txt"), "w") as f:
                f.write(mf.as_parfile(include_info=False))
        print("wrote", name, file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv[1:] or list(PARS))
