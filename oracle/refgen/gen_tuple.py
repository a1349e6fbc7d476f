"""Golden fixture for grid_chisq_derived / tuple_chisq / tuple_chisq_derived (reference
gridutils.py:392, :588, :773) on NGC6440E -- reference run (container only).

The base fitter is the one WLSFitter iteration of gen_ngc6440e.py (its post-fit model is
every grid's starting model).  The derived parameterisation is the reference docstring's
(F0, tau) -> (F0, F1 = -F0 / 2 tau) (gridutils.py:447-452, :832-842), tau in seconds.  All
three run the reference's parallel path (ncpu=2: a deep copy of the fitter per point, a cold
start), which is the semantics the batched GPU grid follows.
"""
import copy

import numpy as np
import astropy.units as u

from refcommon import REFDATA, register_clockless_sites, split_ld, save
import pint.toa as toa
from pint.models import get_model
from pint.fitter import WLSFitter
from pint.gridutils import grid_chisq_derived, tuple_chisq, tuple_chisq_derived


def main():
    register_clockless_sites()
    model = get_model(f"{REFDATA}/NGC6440E.par")
    toas = toa.get_TOAs(f"{REFDATA}/NGC6440E.tim", ephem="builtin", include_bipm=False,
                        planets=False, model=model)
    f = WLSFitter(toas, model)
    f.fit_toas(maxiter=1)
    F0 = np.longdouble(f.model.F0.value)
    F1 = np.longdouble(f.model.F1.value)
    sF0 = np.longdouble(f.model.F0.uncertainty_value)
    sF1 = np.longdouble(f.model.F1.uncertainty_value)
    tau0 = -F0 / (2 * F1)
    arrays, meta = {}, {"name": "grid_tuple"}

    # grid_chisq_derived: 4 F0 values x 3 tau values
    g0 = F0 + np.linspace(-2, 2, 4) * sF0
    gt = tau0 * (1 + np.linspace(-2, 2, 3) * sF1 / -F1)
    arrays["gd_F0_hi"], arrays["gd_F0_lo"] = split_ld(g0)
    arrays["gd_tau_hi"], arrays["gd_tau_lo"] = split_ld(gt)
    fg = WLSFitter(toas, copy.deepcopy(f.model))
    c2, out, ex = grid_chisq_derived(fg, ("F0", "F1"), (lambda x, y: x, lambda x, y: -x / 2 / y),
                                     (g0 * u.Hz, gt * u.s), extraparnames=("DM",), ncpu=2,
                                     printprogress=False)
    arrays["gd_chi2"] = np.asarray(c2, dtype=np.float64)
    arrays["gd_out_F1_hi"], arrays["gd_out_F1_lo"] = split_ld(out[1].to_value(u.Hz / u.s))
    arrays["gd_DM_hi"], arrays["gd_DM_lo"] = split_ld(ex["DM"].to_value(u.pc / u.cm ** 3))

    # tuple_chisq: six (F0, F1) points off the grid's lattice
    a = np.array([-2, -1, 0, 1, 2, 3], dtype=np.longdouble)
    b = np.array([1, -2, 0, 2, -1, 0], dtype=np.longdouble)
    t0, t1 = F0 + a * sF0, F1 + b * sF1
    arrays["tp_F0_hi"], arrays["tp_F0_lo"] = split_ld(t0)
    arrays["tp_F1_hi"], arrays["tp_F1_lo"] = split_ld(t1)
    fg = WLSFitter(toas, copy.deepcopy(f.model))
    c2, ex = tuple_chisq(fg, ("F0", "F1"), [(x * u.Hz, y * u.Hz / u.s) for x, y in zip(t0, t1)],
                         extraparnames=("DM",), ncpu=2, printprogress=False)
    arrays["tp_chi2"] = np.asarray(c2, dtype=np.float64)
    arrays["tp_DM_hi"], arrays["tp_DM_lo"] = split_ld(ex["DM"].to_value(u.pc / u.cm ** 3))

    # tuple_chisq_derived: five (F0, tau) points
    d0 = F0 + np.array([-1, 0, 1, 2, -2], dtype=np.longdouble) * sF0
    dt = tau0 * (1 + np.array([0, 1, -1, 2, -2], dtype=np.longdouble) * sF1 / -F1)
    arrays["td_F0_hi"], arrays["td_F0_lo"] = split_ld(d0)
    arrays["td_tau_hi"], arrays["td_tau_lo"] = split_ld(dt)
    fg = WLSFitter(toas, copy.deepcopy(f.model))
    c2, out, ex = tuple_chisq_derived(fg, ("F0", "F1"), (lambda x, y: x, lambda x, y: -x / 2 / y),
                                      [(x * u.Hz, y * u.s) for x, y in zip(d0, dt)],
                                      extraparnames=("DM",), ncpu=2, printprogress=False)
    arrays["td_chi2"] = np.asarray(c2, dtype=np.float64)
    f1 = np.array([o[1].to_value(u.Hz / u.s) for o in out], dtype=np.longdouble)
    arrays["td_out_F1_hi"], arrays["td_out_F1_lo"] = split_ld(f1)
    arrays["td_DM_hi"], arrays["td_DM_lo"] = split_ld(ex["DM"].to_value(u.pc / u.cm ** 3))
    save("grid_tuple", arrays, meta)


if __name__ == "__main__":
    main()
