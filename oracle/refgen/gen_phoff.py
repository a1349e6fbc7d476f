"""Golden fixtures with an explicit PhaseOffset (PHOFF free; reference run, container only).

* wls_phoff   : the C5 isolated template without red noise, PHOFF free, WLSFitter: residuals
                without the implicit mean subtraction (residuals.py:124-128), the PHOFF
                design-matrix column in place of Offset (timing_model.py:2145), phase
                offset of the non-TZR TOAs (phase_offset.py offset_phase).
* ecorr_phoff : the same with ECORR and no time-correlated noise, four frequencies per epoch:
                the ECORR-only Sherman-Morrison chi2 (residuals.py:591-636, dispatch
                :705-709) and its log-normalisation, GLSFitter.
* phoff_red   : PhaseOffset with PHOFF frozen and PLRedNoise (+ the template's DMX): no
                Offset column in the fit, and the Woodbury chi2 appends the ones column with
                Phi = 1e40 (residuals.py:583-585) -- GLSFitter, DownhillGLSFitter.
* phoff_ecorr : the same with ECORR as well (four frequencies per epoch).
* phoff_dmn   : phoff_red with PLDMNoise beside PLRedNoise: the ones column's row of Sigma
                then includes the DM modes' (1400 MHz / f)^2-scaled weighted sums.
N = 600 TOAs each.  Usage: run_ref.sh gen_phoff.py [name ...]
"""
import io
import os
import sys

import numpy as np
import astropy.units as u

from refcommon import GOLDEN, register_clockless_sites
import pint.simulation as sim
from pint.models import get_model
from gen_synth import pta_par, capture


def par_phoff(seed, ecorr):
    lines = [l for l in pta_par(seed, "").splitlines() if not l.startswith("TNRed")]
    lines.append("PHOFF 0.05 1")
    if ecorr:
        lines.append("ECORR -f fake 0.8")
    return "\n".join(lines) + "\n"


def par_frozen(seed, ecorr, dmn=False):
    lines = pta_par(seed, "").splitlines()  # keeps the template's PLRedNoise
    lines.append("PHOFF 0.05")              # frozen
    if ecorr:
        lines.append("ECORR -f fake 0.8")
    if dmn:  # PLDMNoise (noise_model.py:443), as pta_dmn
        lines += ["TNDMAMP -13.2", "TNDMGAM 2.8", "TNDMC 20"]
    return "\n".join(lines) + "\n"


def gen(name, seed, ecorr, fit, frozen=False, dmn=False):
    np.random.seed(seed)
    par = par_frozen(seed, ecorr, dmn) if frozen else par_phoff(seed, ecorr)
    model = get_model(io.StringIO(par))
    ts = sim.make_fake_toas_uniform(53000, 56652, 600, model,
                                    freq=np.array([800, 1200, 1600, 2000]) * u.MHz,
                                    obs="geocenter", error=0.5 * u.us, add_noise=True,
                                    add_correlated_noise=ecorr or frozen, include_bipm=False,
                                    multi_freqs_in_epoch=ecorr, flags={"f": "fake"})
    model.find_empty_masks(ts, freeze=True)
    if ecorr:
        ne = model.components["EcorrNoise"].get_noise_basis(ts).shape[1]
        print(f"{name}: {ne} ECORR epochs", file=sys.stderr)
        assert ne > 50
    with open(os.path.join(GOLDEN, name + ".par"), "w") as f:
        f.write(par)
    capture(name, model, ts, fit=fit)


if __name__ == "__main__":
    register_clockless_sites()
    which = sys.argv[1:] or ["wls_phoff", "ecorr_phoff"]
    if "wls_phoff" in which:
        gen("wls_phoff", 5, False, "wls")
    if "ecorr_phoff" in which:
        gen("ecorr_phoff", 6, True, "gls")
    if "phoff_red" in which:
        gen("phoff_red", 7, False, "gls", frozen=True)
    if "phoff_ecorr" in which:
        gen("phoff_ecorr", 8, True, "gls", frozen=True)
    if "phoff_dmn" in which:
        gen("phoff_dmn", 9, False, "gls", frozen=True, dmn=True)
