"""Noise-parameter fitting: the likelihood of DownhillFitter._fit_noise
(fitter.py:1230-1273) and its gradients (residuals.py:713-828, noise_model.py:183-214),
evaluated on the device.

The reference maximises Residuals.lnlikelihood() over the free noise parameters with the
residuals of the current timing model held fixed (one Residuals object whose model's noise
values change, fitter.py:1239-1247).  NoiseLikelihood keeps those residuals on the device and
evaluates, per trial point, one of:

* kind 0 -- no correlated noise: diagonal N (residuals.py:638 _calc_wls_chi2);
* kind 1 -- ECORR only with PHOFF free: per-epoch Sherman-Morrison (residuals.py:591);
* kind 2 -- ECORR only without PhaseOffset: as 1 plus the 1e40 offset column of
  _calc_gls_chi2 (residuals.py:583-587);

in one k_noise_lnl pass (pint_noise_lnlike), or

* kind 3 -- time-correlated noise (PLRedNoise): the Woodbury chi2 and logdet of the GLS path
  (pint_fit_step(1) + pint_chi2_gls + pint_lognorm) after pint_set_sigma /
  pint_set_noise_weights put the trial uncertainties and prior variances in place.

TOAs are grouped into white-noise classes (the set of EFAC/EQUAD masks selecting them), so
a trial point uploads one (Q^2, F) pair per class, not n uncertainties.

Gradients (kinds 0 and 1, where the reference defines d_lnlikelihood_d_param): the device
returns sum_i N_i dlnL/dN_i and sum_i dlnL/dN_i per class and dlnL/dw_e per ECORR epoch;
the chain rule to EFAC/EQUAD/ECORR is below.  For ECORR these are the correct derivatives;
the reference's own ECORR branches do not run in this version (d_lnlikelihood_d_Ndiag
squares the ECORR weights that are already variances, residuals.py:741-768, and fails to
broadcast; d_lnlikelihood_d_ECORR raises a UnitConversionError, :779-807 -- recorded in
tests/golden/noise_fit.json), so their parity is pinned by finite differences of the
reference-pinned likelihood.
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L
from .engine import Session, build_layout, pack_table
from .noise import fourier_modes

NOISE_COMPONENTS = ("ScaleToaError", "EcorrNoise", "PLRedNoise", "PLDMNoise")
RED_PARAMS = ("TNREDAMP", "TNREDGAM", "RNAMP", "RNIDX", "TNDMAMP", "TNDMGAM")
KIND_WLS, KIND_ECORR, KIND_ECORR_OFFSET, KIND_WOODBURY = range(4)


def _base(name: str) -> str:
    return name.rstrip("0123456789")


def noise_params(model) -> List[str]:
    """timing_model.get_params_of_component_type("NoiseComponent"), in params order."""
    return [n for n in model.params if model[n].component in NOISE_COMPONENTS]


def free_noise_params(model) -> List[str]:
    """DownhillFitter._get_free_noise_params (fitter.py:1210)."""
    return [n for n in noise_params(model) if not model[n].frozen]


def likelihood_kind(model) -> int:
    """Which branch of Residuals.calc_chi2 (residuals.py:703-711) the model takes."""
    if not model.has_correlated_errors:
        return KIND_WLS
    if model.has_time_correlated_errors:
        return KIND_WOODBURY
    if "PhaseOffset" in model.components:
        if "PHOFF" not in model.free_params:  # residuals.py:595-599 asserts it
            raise ValueError("the ECORR likelihood with a PhaseOffset needs PHOFF free (residuals.py:595-599)")
        return KIND_ECORR
    return KIND_ECORR_OFFSET


def white_noise_classes(model, toas):
    """TOAs grouped by the EFAC/EQUAD masks that select them (first-appearance order):
    (cls_ptr, cls_idx, efac_of_class, equad_of_class)."""
    n = toas.ntoas
    efacs = model.mask_params("EFAC")
    equads = [e for e in model.mask_params("EQUAD") if model[e].value is not None]
    names = efacs + equads
    bits = np.zeros((n, max(len(names), 1)), dtype=bool)
    for j, name in enumerate(names):
        p = model[name]
        bits[toas.select_mask(p.key, p.key_value), j] = True
    _, first, inv = np.unique(bits, axis=0, return_index=True, return_inverse=True)
    inv = np.asarray(inv).ravel()
    order = np.argsort(first, kind="stable")  # class ids by first TOA
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    cls = rank[inv]
    idx = np.argsort(cls, kind="stable").astype(np.int32)
    ptr = np.concatenate([[0], np.cumsum(np.bincount(cls, minlength=len(order)))]).astype(np.int32)
    rows = bits[idx[ptr[:-1]]]
    cls_efac = [[names[j] for j in range(len(efacs)) if r[j]] for r in rows]
    cls_equad = [[names[j] for j in range(len(efacs), len(names)) if r[j]] for r in rows]
    return ptr, idx, cls_efac, cls_equad


class NoiseLikelihood:
    """lnL(noise parameters) of fixed residuals, on the device (fitter.py:1242-1261)."""

    def __init__(self, toas, model, params: Optional[Sequence[str]] = None):
        self.model = copy.deepcopy(model)  # fitter.py:1239 model1: trial values go here
        self.toas = toas
        self.params = list(free_noise_params(model) if params is None else params)
        for name in self.params:
            b = _base(name)
            if name not in self.model._params or not (b in ("EFAC", "EQUAD", "ECORR") or name in RED_PARAMS):
                raise NotImplementedError(f"noise parameter {name} is not fittable on this path")
            if name in RED_PARAMS and self.model[name].value is None:
                raise ValueError(f"{name} has no value")
        self.kind = likelihood_kind(self.model)
        self.ptr, self.idx, self.cls_efac, self.cls_equad = white_noise_classes(self.model, toas)
        self.sigma0 = np.ascontiguousarray(toas.get_errors(), dtype=np.float64)
        self.s = Session()
        try:
            lay = self.s.add(build_layout(self.model, toas, use_gls_basis=self.kind != KIND_WLS))
            self.lay = lay
            self.s.set_instances([(lay, pack_table(lay))])
            self.s.eval(want_M=Session.FIT if self.kind == KIND_WOODBURY else False)
            self.time_resids = self.s.read_resids()[0][0].copy()
            if self.kind != KIND_WOODBURY:
                self.s.set_noise_classes(lay, self.ptr, self.idx, self.sigma0)
        except Exception:
            self.s.close()
            raise
        self._cache = None
        self.nfev = 0

    def close(self):
        self.s.close()

    def set_resids(self, time_resids):
        """Hold other residuals fixed (seconds; e.g. the reference's own, for stage-wise
        parity)."""
        self.s.set_resids([np.asarray(time_resids, dtype=np.float64)])
        self.time_resids = np.array(time_resids, dtype=np.float64)
        self._cache = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- parameter plumbing ------------------------------------------------------------
    def set_values(self, xs):
        for name, x in zip(self.params, xs):
            self.model[name].value = float(x)

    def _qf(self):
        m = self.model
        q2 = [sum(float(m[e].value) ** 2 for e in eqs) for eqs in self.cls_equad]
        f = [float(np.prod([float(m[e].value) for e in efs])) if efs else 1.0 for efs in self.cls_efac]
        return np.column_stack([q2, f])

    def _ep_w(self):
        if self.lay.nep == 0:
            return None
        return np.array([(float(self.model[p].value) * 1e-6) ** 2 for p in self.lay.ep_param])

    def sigma_us(self):
        """Scaled uncertainties at the current values (noise_model.py:159 scale_toa_sigma)."""
        qf = self._qf()
        sg = np.empty(self.lay.n)
        for c in range(len(qf)):
            rows = self.idx[self.ptr[c]:self.ptr[c + 1]]
            sg[rows] = np.hypot(self.sigma0[rows], np.sqrt(qf[c, 0])) * qf[c, 1]
        return sg

    # -- evaluation --------------------------------------------------------------------
    def evaluate(self, xs, grad=True):
        """(lnL, chi2, logdet C / 2, gradient or None) at the free values xs."""
        key = tuple(float(x) for x in xs)
        if self._cache is None or self._cache[0] != key:
            self.set_values(xs)
            self.nfev += 1
            if self.kind == KIND_WOODBURY:
                res = self._eval_woodbury()
            else:  # the gradient sums come from the same pass
                want = self.kind in (KIND_WLS, KIND_ECORR)
                out, g, eg = self.s.noise_lnlike([self.kind], self._qf(), self._ep_w(), grad=want)
                res = (float(out[0, 0]), float(out[0, 1]), float(out[0, 2]), self._chain(g, eg) if want else None)
            self._cache = (key, res)
        return self._cache[1]

    def _eval_woodbury(self):
        s, lay = self.s, self.lay
        s.set_sigma(lay, self.sigma_us() * 1e-6)
        red = fourier_modes(self.model, self.toas)[1] if lay.nred > 0 else None
        s.set_noise_weights(lay, red, self._ep_w())
        try:  # only the Woodbury factor of the noise block is needed (cf. Residuals.update)
            s.fit_step(1)
        except L.PintError as e:
            if e.code != L.PINT_E_NOT_PD:
                raise
        chi2 = float(s.chi2_gls()[0])
        ln = float(s.lognorm(1)[0])
        return -(0.5 * chi2 + ln), chi2, ln, None

    def _chain(self, g, eg):
        """dlnL/dparam from the per-class / per-epoch sums (residuals.py:772-828 with
        noise_model.py:183-214): dN_i/dEFAC_p = 2 N_i / EFAC_p, dN_i/dEQUAD_p =
        2 EQUAD_p F_c^2 (us^2 -> s^2), dw_e/dECORR_p = 2 ECORR_p (us^2 -> s^2)."""
        m = self.model
        qf = self._qf()
        out = np.zeros(len(self.params))
        for k, name in enumerate(self.params):
            b = _base(name)
            v = float(m[name].value)
            if b == "EFAC":
                out[k] = sum(2.0 * g[c, 0] / v for c, efs in enumerate(self.cls_efac) if name in efs)
            elif b == "EQUAD":
                out[k] = sum(2.0 * v * qf[c, 1] ** 2 * 1e-12 * g[c, 1]
                             for c, eqs in enumerate(self.cls_equad) if name in eqs)
            elif b == "ECORR":
                out[k] = sum(2.0 * v * 1e-12 * eg[e] for e, p in enumerate(self.lay.ep_param or []) if p == name)
            else:
                raise NotImplementedError(f"d_lnlikelihood_d_param is not defined for parameter {name}.")
        return out

    def lnlikelihood(self, xs=None) -> float:
        if xs is None:
            xs = [self.model[p].value for p in self.params]
        return self.evaluate(xs, grad=False)[0]

    def d_lnlikelihood_d_params(self, xs=None) -> np.ndarray:
        """residuals.py:809-828 d_lnlikelihood_d_param for every free parameter; raises
        NotImplementedError where the reference does (correlated noise without PHOFF free,
        or time-correlated noise)."""
        if self.kind not in (KIND_WLS, KIND_ECORR):
            raise NotImplementedError
        if xs is None:
            xs = [self.model[p].value for p in self.params]
        return self.evaluate(xs, grad=True)[3]


def hessian(f, x, rel=1e-3, floor=1e-1):
    """Central-difference Hessian with one Richardson extrapolation (steps h and h/2,
    h_i = rel * max(|x_i|, floor)).  Replaces numdifftools.Hessian (fitter.py:1270), which
    is not available on this image; the uncertainties it yields are therefore pinned by the
    closed-form Hessian of a one-EFAC likelihood (tests/test_noise_fit.py), not by the
    reference."""
    x = np.asarray(x, dtype=np.float64)
    n = len(x)
    f0 = f(x)

    def at(h):
        H = np.zeros((n, n))
        for i in range(n):
            e = np.zeros(n)
            e[i] = h[i]
            H[i, i] = (f(x + e) - 2.0 * f0 + f(x - e)) / h[i] ** 2
            for j in range(i):
                d = np.zeros(n)
                d[j] = h[j]
                H[i, j] = H[j, i] = (f(x + e + d) - f(x + e - d) - f(x - e + d) + f(x - e - d)) / (4.0 * h[i] * h[j])
        return H

    h = rel * np.maximum(np.abs(x), floor)
    return (4.0 * at(h / 2) - at(h)) / 3.0


def fit_noise(toas, model, noisefit_method="Newton-CG", uncertainty=False):
    """DownhillFitter._fit_noise (fitter.py:1230-1273): maximise lnL over the free noise
    parameters, Newton-CG with the analytic gradient without correlated noise, Nelder-Mead
    with it; (values, errors) with uncertainty=True, errors = sqrt(diag(pinv(Hessian)))."""
    import scipy.optimize as opt

    nl = NoiseLikelihood(toas, model)
    try:
        xs0 = [float(model[p].value) for p in nl.params]

        def _mloglike(xs):
            return -nl.evaluate(xs, grad=False)[0]

        if not model.has_correlated_errors:
            def _mloglike_grad(xs):
                return -nl.evaluate(xs, grad=True)[3]

            res = opt.minimize(_mloglike, xs0, method=noisefit_method, jac=_mloglike_grad)
        else:
            res = opt.minimize(_mloglike, xs0, method="Nelder-Mead")
        if uncertainty:
            H = hessian(_mloglike, res.x)
            errs = np.sqrt(np.diag(np.linalg.pinv(H)))
            return res.x, errs
        return res.x
    finally:
        nl.close()
