"""Fitter.get_summary (reference fitter.py:348-472) and the value(uncertainty) shorthand it
prints fitted parameters with.

The reference formats a fitted parameter as ``format(ufloat(value, unc), "28SP")`` with the
``uncertainties`` package (absent on this image).  ``shorthand`` restates that package's
published rules for the default precision: the uncertainty keeps the significant digits of
the Particle Data Group rule (its leading three digits 100-354: two digits, 355-949: one,
950-999: rounded up to two digits of the next power of ten), the value is rounded to the
uncertainty's last digit, and the uncertainty is written as an integer in units of that
digit in parentheses; ``P`` prints a common exponent as ``×10⁻⁵``.  A common exponent is used
when the value's (or a larger uncertainty's) decimal exponent is below -4 or the digits
would reach beyond the units position of a fixed-point form, as for Python's ``g``.
"""
from __future__ import annotations

import math

import numpy as np

_SUP = str.maketrans("0123456789-+", "⁰¹²³⁴⁵⁶⁷⁸⁹⁻⁺")


def _pdg_digits(unc):
    """(number of significant digits, exponent of the uncertainty after rounding)."""
    e = math.floor(math.log10(unc))
    d3 = int(round(unc / 10.0 ** (e - 2)))
    if d3 >= 1000:  # rounding carried into the next decade
        e += 1
        d3 //= 10
    if d3 <= 354:
        return 2, e
    if d3 <= 949:
        return 1, e
    return 2, e + 1


def shorthand(value, unc, pretty=True):
    """``value(unc)`` as uncertainties formats ``ufloat(value, unc)`` with ``SP`` (or ``S``)."""
    value = np.longdouble(value)  # longdouble parameters keep their digits (F0, PB, ...)
    if unc is None or not np.isfinite(unc) or unc <= 0:
        return f"{float(value):g}"
    unc = float(unc)
    nsig, eu = _pdg_digits(unc)
    last = eu - nsig + 1                      # decimal position of the last shown digit
    ref = max(abs(float(value)), unc)
    ev = math.floor(math.log10(ref)) if ref > 0 else eu
    use_exp = ev < -4 or (last > 0 and ev >= 6)
    v, last_s = (value / np.longdouble(10) ** ev, last - ev) if use_exp else (value, last)
    ui = int(round(unc / 10.0 ** last))
    if last_s <= 0:
        vs = np.format_float_positional(v, precision=-last_s, unique=False, fractional=True, trim="k")
        if last_s == 0:
            vs = vs.rstrip(".")
        us = f"{ui}"
    else:  # the uncertainty's last digit left of the units digit: both in full
        q = np.longdouble(10) ** last_s
        vs = np.format_float_positional(np.round(v / q) * q, precision=0, unique=False, trim="-")
        us = f"{ui * 10 ** last_s}"
    s = f"{vs}({us})"
    if use_exp:
        s = f"{s}×10{str(ev).translate(_SUP)}" if pretty else f"{s}e{ev:+03d}"
    return s


def _fmt_angle(p, value):
    """Sexagesimal string of an angle parameter (hh:mm:ss / dd:mm:ss)."""
    if value is None:
        return ""
    v = float(value)
    sign = "-" if v < 0 else ""
    v = abs(v)
    a = int(v)
    m = int((v - a) * 60)
    sec = (v - a - m / 60.0) * 3600.0
    unit = ("h", "m", "s") if p.kind == "hourangle" else ("d", "m", "s")
    return f"{sign}{a}{unit[0]}{m:02d}{unit[1]}{sec:011.8f}{unit[2]}"


def _num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def fitter_summary(f, nodmx=False):
    m, m0 = f.model, f.model_init
    wb = getattr(f, "is_wideband", False)
    s = (f"Fitted model using {f.method} method with {len(m.free_params)} free parameters to "
         f"{f.toas.ntoas} TOAs\n")
    if wb:
        s += (f"Prefit TOA residuals Wrms = {f.resids_init.toa.rms_weighted()} us, Postfit TOA residuals Wrms = "
              f"{f.resids.toa.rms_weighted()} us\n")
        s += (f"Prefit DM residuals Wrms = {f.resids_init.dm.rms_weighted()} pc / cm3, Postfit DM residuals Wrms = "
              f"{f.resids.dm.rms_weighted()} pc / cm3\n")
    else:
        s += (f"Prefit residuals Wrms = {f.resids_init.rms_weighted()} us, Postfit residuals Wrms = "
              f"{f.resids.rms_weighted()} us\n")
    s += (f"Chisq = {f.resids.chi2:.3f} for {f.resids.dof} d.o.f. for reduced Chisq of "
          f"{f.resids.reduced_chi2:.3f}\n\n")
    names = [pn for pn in m.params if not (nodmx and pn.startswith("DMX"))]
    w = max((len(pn) for pn in names), default=0)
    sp = str(w)
    s += ("{:<" + sp + "s} {:^20s} {:^28s} {}\n").format("PAR", "Prefit", "Postfit", "Units")
    s += ("{:<" + sp + "s} {:>20s} {:>28s} {}\n").format("=" * w, "=" * 20, "=" * 28, "=" * 5)
    for pn in names:
        par = m[pn]
        pre = m0[pn] if pn in m0 else None
        pv = pre.value if pre is not None else None
        if par.value is None:
            continue
        if par.kind in ("str",):
            s += ("{:" + sp + "s} {:>20s} {:28s} {}\n").format(pn, "" if pv is None else str(pv), str(par.value),
                                                                par.units)
        elif par.kind in ("hourangle", "degangle"):
            if par.frozen:
                s += ("{:" + sp + "s} {:>20s} {:>28s} {} \n").format(pn, _fmt_angle(par, pv), "", par.units)
            else:
                # uncertainty in seconds of time (hourangle) or arcseconds (pint.hourangle_second / u.arcsec)
                unc = (par.uncertainty or 0.0) * 3600.0
                uu = "hourangle_second" if par.kind == "hourangle" else "arcsec"
                s += ("{:" + sp + "s} {:>20s}  {:>16s} +/- {:.2g} {}\n").format(
                    pn, _fmt_angle(par, pv), _fmt_angle(par, par.value), unc, uu)
        elif par.kind == "bool":
            s += ("{:" + sp + "s} {:>20s} {:28s} {}\n").format(pn, "Y" if pv else "N", "", par.units)
        elif par.frozen:
            v, p0 = _num(par.value), _num(pv)
            if pn in ("START", "FINISH", "CHI2", "CHI2R", "TRES", "DMRES"):
                if p0 is None:
                    s += ("{:" + sp + "s} {:20s} {:28g} {} \n").format(pn, " ", v, par.units)
                else:
                    s += ("{:" + sp + "s} {:20g} {:28g} {} \n").format(pn, p0, v, par.units)
            else:
                s += ("{:" + sp + "s} {:20g} {:28s} {} \n").format(pn, p0 if p0 is not None else 0.0, "", par.units)
        else:
            s += ("{:" + sp + "s} {:20g} {:>28s} {} \n").format(
                pn, _num(pv) if pv is not None else 0.0, shorthand(par.value, par.uncertainty), par.units)
    return s
