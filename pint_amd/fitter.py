"""Fitters (host mirror of reference fitter.py): WLSFitter (:1940), GLSFitter (:2090),
DownhillWLSFitter (:1379), DownhillGLSFitter (:1527), Fitter.auto (:252).

The numerical work -- design matrix, residuals, Gram on FP64 MFMA, Cholesky, step,
covariance, Woodbury chi2, parameter update in double-double -- runs on the GPU; the host
only sequences launches and applies the reference's control flow (downhill lambda halving
and convergence rules, exceptions).  ``BatchFit`` drives many independent fits (grid
points, PTA pulsars) through one launch sequence per iteration.
"""
from __future__ import annotations

import copy
import warnings
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L
from .engine import Session, build_layout, pack_table, unpack_table
from .pint_matrix import CorrelationMatrix, CovarianceMatrix  # noqa: F401  (re-exported)


class ConvergenceFailure(ValueError):
    pass


class MaxiterReached(ConvergenceFailure):
    pass


class StepProblem(ConvergenceFailure):
    pass


class CorrelatedErrors(ValueError):
    def __init__(self, model):
        super().__init__(f"Model has correlated errors and requires a GLS-based fitter: {model}")


class InvalidModelParameters(ValueError):
    pass


class DegeneracyWarning(UserWarning):
    pass


class FitResult:
    """Per-instance fit outcome of a BatchFit."""

    def __init__(self):
        self.chi2 = np.nan
        self.errors = None
        self.cov = None
        self.converged = False
        self.status = "ok"
        self.noise_coeffs = None
        self.noise_resids = {}
        self.fac = None     # the design-matrix normalisation of the step (Fitter.fac)
        self.step = None    # the parameter step, timing columns (par units)


class BatchOutcome:
    """Per-instance fit outcomes as arrays (BatchFit with outputs=False, grid points)."""

    def __init__(self, chi2, converged, exc):
        self.chi2 = chi2
        self.converged = converged
        self.step_problem = exc
        self.maxiter_reached = ~converged & ~exc


def model_key(model, freeze=()):
    """Everything a pulsar upload (build_layout) depends on besides the TOAs: every
    parameter's name, value and frozen flag (noise values set sigma and the basis weights,
    the frozen set the columns) and the component set.  freeze: parameters keyed as frozen
    whatever their flag (the model a grid would copy and freeze them in)."""
    return (tuple((n, str(model[n].value), bool(model[n].frozen) or n in freeze) for n in model.params),
            tuple(model.components), model.binary)


class BatchFit:
    """Run the same fitter on many (model, toas) instances at once.

    mode: 'wls' | 'gls'; downhill: reference DownhillFitter control flow per instance.
    Each instance's model is updated in place at the end (like fitter.model).

    Instances are independent: an instance whose evaluation raises an invalid-parameter
    status (ECC outside [0, 1), a Kepler solve that does not converge, ...) fails alone.  At
    a state the fit has to stand on (the initial model, or the result of a plain step) it is
    taken out of the device batch and reported as failed (chi2 NaN, status
    "InvalidModelParameters"; fitter.py:926-935 raises InvalidModelParameters for that fit
    only, gridutils.py:89-106 returns NaN for that point); at a downhill trial state it
    counts as a rejected trial, so that instance halves its lambda (fitter.py:1040-1057).
    """

    EVAL_ERRORS = (L.PINT_E_KEPLER, L.PINT_E_PARAM)

    def __init__(self, items: Optional[Sequence[tuple]], mode: str = "wls", session: Optional[Session] = None,
                 layouts=None, tables=None, threshold=None, degeneracy_style=None, track_mode=None,
                 wideband=False, want_fac=False, fac_style=None, own_session=None, grid=None):
        """items: [(model, toas)], or None with `layouts` + `tables` given (instances that
        are bare parameter tables of already-uploaded pulsars, e.g. grid points).

        threshold: the SVD cut of the reference fitter (fitter.py:1314 WLS: None ->
        1e-14 max(N, P); GLS: 0); used when the normal equations are degenerate.
        degeneracy_style: the DegeneracyWarning text of "wls" (WLSState), "gls"
        (GLSFitter) or "glsstate" (GLSState, the downhill GLS fitter).
        grid: (layout, base table, variables, npts, k0) -- grid points whose tables are formed
        on the device (Session.set_grid) instead of `tables`."""
        self.items = list(items) if items is not None else None
        self.mode = mode
        self.want_fac = bool(want_fac)  # read the step's normalisation back (Fitter.fac)
        self.fac_style = fac_style      # None | "timing" | "wbstate" (_fac_into)
        # a Session passed in belongs to the caller (a resident upload, a grid session)
        self.own_session = (session is None) if own_session is None else bool(own_session)
        self.threshold = threshold
        self.degeneracy_style = degeneracy_style or mode
        self.degenerate = None  # per instance: dropped directions of the last SVD-path step
        self.gls = mode == "gls"
        self.s = session or Session()
        self.grid = grid
        if grid is not None:
            layouts = [grid[0]] * int(grid[3])
            tables = None
        if layouts is None:
            layouts = []
            cache = {}
            for model, toas in self.items:
                key = (id(toas), model_key(model))
                if key in cache:
                    layouts.append(cache[key])
                    continue
                lay = self.s.add(build_layout(model, toas, track_mode=track_mode, use_gls_basis=self.gls))
                cache[key] = lay
                layouts.append(lay)
        if tables is None and grid is None:
            tables = [pack_table(l, m) for l, (m, _) in zip(layouts, self.items)]
        self.n0 = len(layouts)
        self.idx = np.arange(self.n0)                 # device instance -> original index
        self.failed = np.zeros(self.n0, dtype=bool)  # original instances taken out of the batch
        self.tables0 = tables
        self.grid_like = grid is not None or (isinstance(tables, np.ndarray) and tables.ndim == 2 and len(layouts) > 0
                                              and len(set(map(id, layouts))) == 1)  # one layout object (C-level scan)
        self.layouts0 = layouts if grid is not None else list(layouts)  # (a grid's list is its own)
        self._bind(list(layouts), tables)
        # wideband (WidebandTOAFitter / WidebandDownhillFitter): the DM rows join every fit
        # step (k_wb_gram) and every chi2 (the DM chi2 of WidebandTOAResiduals)
        self.wideband = bool(wideband)
        if self.wideband:
            for lay in {id(l): l for l in layouts}.values():
                if self.s.fit_layout(lay)[0] != 1:
                    raise NotImplementedError("wideband fits on the device need the compact DMX layout (>= 8 "
                                              "free DMX bins, no TOA in two free bins, no ECORR)")
                self.s.set_wideband(lay)
            self.s.set_wbfit(True)

    def _bind(self, layouts, tables):
        self.layouts = layouts
        if self.grid is not None and tables is None:
            lay, base, variables, npts, k0 = self.grid
            self.s.set_grid(lay, base, variables, npts, k0)  # the points' tables formed on the device
        elif self.grid_like:
            self.s.set_instances_of(layouts[0], np.asarray(tables).reshape(len(layouts), -1))  # grid points
        else:
            self.s.set_instances(list(zip(layouts, tables)))
        self.ninst = len(layouts)
        # (an array: a grid's 65,536-point Python list took ~0.1 ms per any() / np.where)
        if self.grid_like and layouts:
            self.use_gls_chi2 = np.full(len(layouts), self.gls and (layouts[0].nred > 0 or layouts[0].nep > 0))
        else:
            self.use_gls_chi2 = np.array([self.gls and (l.nred > 0 or l.nep > 0) for l in layouts], dtype=bool)

    def _drop(self, bad):
        """Take the device instances flagged in `bad` out of the batch (their current tables
        are kept for the others, which are re-bound unchanged)."""
        tabs = self.s.read_tables()
        keep = ~bad
        self.failed[self.idx[bad]] = True
        self.idx = self.idx[keep]
        lays = [l for l, k in zip(self.layouts, keep) if k]
        tabs = [t for t, k in zip(tabs, keep) if k]
        if not lays:
            self.ninst = 0
            raise InvalidModelParameters("every instance of the batch landed at an invalid point")
        self._bind(lays, np.stack(tabs) if self.grid_like else tabs)
        return keep

    def _eval(self, want_M):
        """pint_eval; instances that raise an invalid-parameter status are dropped (their
        evaluation failed at a state the fit cannot leave) and the others re-evaluated.
        Returns the keep mask over the device instances before the call, or None."""
        try:
            self.s.eval(want_M=want_M)
            return None
        except L.PintError as e:
            if e.code not in self.EVAL_ERRORS or self.s.lazy:
                raise
            bad = self.s.inst_status() != 0
            if not bad.any():
                raise
        keep = self._drop(bad)
        self.s.eval(want_M=want_M)
        return keep

    # -- helpers ------------------------------------------------------------------------
    def _chi2_now(self):
        c2, _ = self._chi2_enqueue()()
        if self.wideband:  # WidebandTOAResiduals.chi2 = the TOA chi2 + the DM chi2 (residuals.py:1206)
            c2 = c2 + self.s.dm_resids()[1]
        return c2, None

    def _chi2_enqueue(self):
        """Enqueue the chi2 reads of the current residuals; returns a function giving the
        per-instance chi2 (after check() in lazy mode, where the reads land in pinned
        buffers)."""
        if self.use_gls_chi2.all():
            cg = self.s.chi2_gls()
            return lambda: (np.array(cg, dtype=np.float64), None)
        cw = self.s.read_chi2()
        cg = self.s.chi2_gls() if self.use_gls_chi2.any() else None
        if cg is None:
            return lambda: (np.array(cw, dtype=np.float64), None)
        return lambda: (np.where(self.use_gls_chi2, cg, cw), None)

    def _step(self):
        keep = self._eval(Session.FIT)
        try:
            self.s.fit_step(1 if self.gls else 0)
        except L.PintError as e:
            if e.code != L.PINT_E_NOT_PD or self.s.lazy:
                raise
            self._svd_step()
        return keep

    def _thresholds(self):
        if self.threshold is not None:
            return np.full(self.ninst, float(self.threshold))
        if self.gls:
            return np.zeros(self.ninst)
        return np.array([1e-14 * max(l.n, len(l.columns)) for l in self.layouts])

    def _svd_step(self):
        """Degenerate normal equations: the reference's SVD path (fitter.py:1282-1359 WLS,
        :2196-2230 GLSFitter, :1477-1500 GLSState) on the device (k_eig): directions with
        singular values <= threshold * s_max are dropped, each reported as a
        DegeneracyWarning with the reference's wording."""
        th = self._thresholds()
        dirs = self.s.solve_eig(1 if self.gls else 0, th)
        self.degenerate = dirs
        for k, (lay, vs) in enumerate(zip(self.layouts, dirs)):
            params = list(lay.columns)
            t = th[k]
            for v in vs:
                pairs = list(zip(v[:len(params)], params))
                if self.degeneracy_style == "wls":
                    comb = " + ".join(f"{co}*{p}" for (co, p) in sorted(pairs) if abs(co) > t)
                    msg = f"Parameter degeneracy; the following linear combination yields almost no change: {comb}"
                elif self.degeneracy_style == "glsstate":
                    comb = " ".join(f"{p}" for (co, p) in sorted(pairs) if abs(co) > t)
                    msg = ("Parameter degeneracy; the following combination of parameters yields almost no "
                           f"change: {comb}")
                else:
                    comb = " ".join(f"{co}*{p}" for (co, p) in reversed(sorted(pairs)) if abs(co) > t)
                    msg = ("Parameter degeneracy; the following combination of parameters yields almost no "
                           f"change: {comb}")
                warnings.warn(msg, DegeneracyWarning)

    def _finish(self, results):
        tabs = self.s.read_tables()
        self.final_tables = tabs
        if self.items is not None:
            for k, t in zip(self.idx, tabs):
                m = self.items[k][0]
                unpack_table(self.layouts0[k], t, m)
        for k in np.where(self.failed)[0]:
            results[k].status = "InvalidModelParameters"
            results[k].chi2 = np.nan
        return results

    def _errors_into(self, results):
        dp, er, cov, cl = self.s.read_step()
        self.last_chi2_lin = cl  # the steps' linearised chi2 (WidebandTOAFitter returns it)
        for d, (k, lay) in enumerate(zip(self.idx, self.layouts)):
            res = results[k]
            nc = len(lay.columns)
            res.errors = er[d][:nc].copy()
            res.cov = cov[d].copy()
            res.noise_coeffs = dp[d][nc:lay.K].copy()
            res.step = dp[d][:nc].copy()
            res.labels = list(lay.columns)
            if self.items is not None:
                m = self.items[k][0]
                for j, name in enumerate(lay.columns):
                    if name != "Offset":
                        m[name].uncertainty = float(res.errors[j])

    def _fac_into(self, results):
        """The normalisation of the last step's design matrix per instance (the reference's
        ``fac`` / ``norm``, utils.py:2879 normalize_designmatrix, zero norm -> 1): WLS, the
        column norms of the whitened M (fitter.py:1320-1343); GLS, the column norms of
        [M | noise bases] (fitter.py:2164-2176), with the ECORR quantisation columns
        (sqrt of each epoch's TOA count) after the timing columns and before the Fourier
        bases, the reference's noise_model_designmatrix order.  From the device
        (pint_read_norms: the Gram's diagonal, or the unweighted column sums of squares).
        fac_style "timing": the timing columns only (GLSFitter full_cov=True appends no
        noise basis, fitter.py:2166); "wbstate": WidebandState's norm[ntmpar:] = 1 with
        ntmpar = free parameters + 1 (fitter.py:1652-1657)."""
        if not self.want_fac:
            return
        for nq, k, lay in zip(self.s.read_norms(1 if self.gls else 0), self.idx, self.layouts):
            nc = len(lay.columns)
            if self.gls:
                f = np.sqrt(np.asarray(nq[:lay.K], dtype=np.float64))
                if lay.nep > 0:
                    ep = np.sqrt(np.diff(np.asarray(lay.ep_ptr)).astype(np.float64))
                    f = np.concatenate([f[:nc], ep, f[nc:]])
                if self.fac_style == "timing":
                    f = f[:nc]
                elif self.fac_style == "wbstate":
                    m = self.items[k][0] if self.items is not None else lay.model
                    f[len(m.free_params) + 1:] = 1.0
            else:
                f = np.sqrt(np.asarray(nq[:nc], dtype=np.float64))
            f[f == 0] = 1.0
            results[k].fac = f

    def _noise_into(self, results):
        """Noise realisations of the last step (GLS only)."""
        if not self.gls:
            return
        for k, nr in zip(self.idx, self.s.noise_resids()):
            results[k].noise_resids = nr

    def _full(self, arr, fill):
        arr = np.asarray(arr)
        out = np.full(self.n0, fill, dtype=arr.dtype)
        out[self.idx] = arr
        return out

    # -- plain WLS/GLS (fitter.py:1965-2087, :2104-2289) -------------------------------
    def fit_plain(self, maxiter=1, outputs=True):
        """outputs=False (grid points): no per-instance FitResult, no step/covariance
        read-back; returns a BatchOutcome of arrays (chi2, status)."""
        results = [FitResult() for _ in range(self.n0)] if outputs else None
        for _ in range(maxiter):
            self._step()
            if outputs:
                self._errors_into(results)
                self._fac_into(results)
                self._noise_into(results)
            self.s.apply_step_uniform(1.0)
        self._eval(False)
        c2, _ = self._chi2_now()
        if not outputs:
            chi2 = self._full(np.array(c2, dtype=np.float64), np.nan)
            return self._finish_arrays(chi2, ~self.failed, np.zeros(self.n0, dtype=bool))
        for k, c in zip(self.idx, c2):
            results[k].chi2 = float(c)
            results[k].converged = True
        return self._finish(results)

    def _finish_arrays(self, chi2, converged, exc):
        # the final parameter tables stay on the device until asked for (final_tables_flat)
        out = BatchOutcome(chi2, converged, exc)
        out.failed = self.failed.copy()
        out.maxiter_reached &= ~self.failed
        return out

    def final_tables_flat(self):
        """The instances' parameter tables after the fit, concatenated (device -> host);
        instances taken out of the batch (failed) are NaN."""
        t = self.s.read_tables()
        out = [None] * self.n0
        for k, tt in zip(self.idx, t):
            out[k] = tt
        for k in range(self.n0):
            if out[k] is None:
                out[k] = np.full(self.layouts0[k].tstride, np.nan)
        return np.concatenate(out)

    # -- downhill (fitter.py:999-1105) ---------------------------------------------------
    def fit_downhill(self, maxiter=10, required_chi2_decrease=1e-2, max_chi2_increase=1e-2, min_lambda=1e-3,
                     outputs=True):
        """The reference's per-fitter control flow (fitter.py:1015-1095), applied to every
        instance at once: a lambda-halving line search on each instance's chi2, with the
        best state tracked per instance.  Decisions are vectorised over instances; each
        trial is one batched eval + chi2 of all instances.  A trial state whose evaluation
        fails (invalid parameters) is a rejected trial of that instance only.

        The states stay on the device: the current states are a device snapshot of the
        tables (pint_save_tables), a trial is snapshot + lambda x step (pint_restore_tables,
        k_apply), and an instance that has accepted its step keeps that lambda in the
        following trials of the same iteration, so that after the last trial the tables hold
        every instance's new current state.  Only the chi2 of a trial crosses to the host.
        A state better than an instance's best is always an accepted one (its chi2 is below
        the current state's), so the best tables are read back at most once per iteration."""
        self._step()                                     # step of the initial state (drops invalid ones)
        n = self.ninst
        single = n == 1
        self.s.save_tables()                             # the current states
        best_tab = self.s.read_tables_flat()
        sizes = np.array([l.tstride for l in self.layouts])
        ent = np.repeat(np.arange(n), sizes)             # instance of every table entry
        self._eval(False)
        cur_chi2, _ = self._chi2_now()
        cur_chi2 = np.array(cur_chi2, dtype=np.float64)
        best_chi2 = cur_chi2.copy()
        best_cur = np.ones(n, dtype=bool)                # the best state is the current one
        active = np.ones(n, dtype=bool)
        converged = np.zeros(n, dtype=bool)
        exc = np.zeros(n, dtype=bool)
        for it in range(maxiter):
            if not active.any():
                break
            lam = np.ones(n)
            decided = ~active
            acc_lam = np.zeros(n)                        # the lambda an instance ends the iteration at
            dec = np.zeros(n)
            newbest = np.zeros(n, dtype=bool)
            while not decided.all():
                # one trial: enqueued lazily (restore, lambda x step, evaluation, chi2) and
                # synchronised once; an instance whose evaluation raised a status is a rejected
                # trial (wideband: the DM chi2 read is synchronous, so the trial is too)
                lazy = not self.wideband
                if lazy:
                    self.s.set_lazy(True)
                try:
                    self.s.restore_tables()
                    applied = np.where(decided, acc_lam, lam)
                    if single:
                        self.s.apply_step_uniform(float(applied[0]))
                    else:
                        self.s.apply_step(applied)
                    bad = np.zeros(n, dtype=bool)
                    got = None  # this trial's enqueued chi2 (never a previous trial's)
                    try:
                        self.s.eval(want_M=False)
                        if lazy:
                            got = self._chi2_enqueue()
                            self.s.check()
                            new_chi2, _ = got()
                        else:
                            new_chi2, _ = self._chi2_now()
                    except L.PintError as e:
                        if e.code not in self.EVAL_ERRORS:
                            raise
                        if lazy:  # status and chi2 read synchronously from here on
                            self.s.set_lazy(False)
                            lazy = False
                        bad = self.s.inst_status() != 0
                        if not bad.any():
                            raise
                        # the chi2 enqueued before the error (check() has synchronised it),
                        # else recomputed synchronously
                        new_chi2, _ = got() if got is not None else self._chi2_now()
                finally:
                    if lazy:
                        self.s.set_lazy(False)
                new_chi2 = np.where(bad, np.nan, np.array(new_chi2, dtype=np.float64))
                und = ~decided
                d = cur_chi2 - new_chi2
                ok = np.isfinite(new_chi2)
                better = und & ok & (new_chi2 < best_chi2)          # fitter.py:1046-1049
                best_chi2[better] = new_chi2[better]
                newbest |= better
                bad = und & (~ok | (d < -max_chi2_increase))         # :1050-1062 halve lambda
                lam[bad] /= 2
                gone = bad & (lam < min_lambda)                      # :1058 StepProblem
                exc |= gone
                decided |= gone
                dec[gone] = 0.0
                good = und & ~bad                                    # :1063-1067 accept
                acc_lam[good] = lam[good]
                cur_chi2[good] = new_chi2[good]
                dec[good] = d[good]
                decided |= good
                best_cur[good] = better[good]
            # the tables hold every instance's last trial; its new current state is the
            # accepted lambda (0 after a failed search): re-applied only where they differ,
            # then the snapshot the next iteration's trials start from
            if not np.array_equal(applied, acc_lam):
                self.s.restore_tables()
                if single:
                    self.s.apply_step_uniform(float(acc_lam[0]))
                else:
                    self.s.apply_step(acc_lam)
            self.s.save_tables()
            if newbest.any():
                tab = self.s.read_tables_flat()
                sel = newbest[ent]
                best_tab[sel] = tab[sel]
            done = active & exc
            conv = active & ~exc & (-max_chi2_increase <= dec) & (dec < required_chi2_decrease) & (lam == 1)
            converged |= conv                                        # :1076-1085
            active &= ~(done | conv)
            if active.any() and it < maxiter - 1:
                # step at the new current states (inactive ones are ignored); every current
                # state has been evaluated, so nothing can be dropped here
                if self._step() is not None:
                    raise RuntimeError("a downhill state evaluated before failed its re-evaluation")
        # best state -> model, residuals; covariance from a step at the best state
        if not best_cur.all():
            self.s.set_tables(best_tab)
        if self._step() is not None:
            raise RuntimeError("a downhill best state evaluated before failed its re-evaluation")
        results = None
        if outputs:
            results = [FitResult() for _ in range(self.n0)]
            self._errors_into(results)
            self._fac_into(results)
            self._noise_into(results)
        self.s.eval(want_M=False)
        c2, _ = self._chi2_now()
        if not outputs:
            return self._finish_arrays(self._full(np.array(c2, dtype=np.float64), np.nan),
                                       self._full(converged, False), self._full(exc, False))
        for d, k in enumerate(self.idx):
            r = results[k]
            r.chi2 = float(c2[d])
            r.converged = bool(converged[d])
            r.status = "StepProblem" if exc[d] else ("converged" if converged[d] else "MaxiterReached")
        return self._finish(results)

    def close(self):
        if self.own_session:
            self.s.close()


# ----------------------------------------------------------------------------------
# single-model fitters (reference API)
# ----------------------------------------------------------------------------------
class FitState:
    """The state a fit ended at (the reference's ModelState, fitter.py:908-979, as far as a
    finished fit exposes it: DownhillFitter.current_state, fitter.py:1075): the model and its
    residuals, chi2, the step's design-matrix normalisation ``fac``, the step, the fitted
    columns and their covariance.  The device computed all of it; nothing is re-evaluated."""

    def __init__(self, fitter, model, resids, res):
        self.fitter = fitter
        self.model = model
        self.resids = resids
        self.chi2 = res.chi2
        self.fac = res.fac
        self.norm = res.fac
        self.params = list(res.labels) if getattr(res, "labels", None) is not None else []
        self.step = res.step
        self.noise_ampls = res.noise_coeffs
        self.parameter_covariance_matrix = (CovarianceMatrix(res.cov, res.labels)
                                            if res.cov is not None else None)

    @property
    def covariance_matrix(self):
        warnings.warn("This parameter is deprecated.  Use `parameter_covariance_matrix` instead of "
                      "`covariance_matrix`", DeprecationWarning)
        return self.parameter_covariance_matrix


class Fitter:
    def __init__(self, toas, model, track_mode=None, residuals=None):
        self.toas = toas
        self.model_init = model
        self.track_mode = track_mode
        self.model = copy.deepcopy(model)
        self._resids_init = residuals
        self.resids = None
        self.converged = False
        self.method = None
        self.is_wideband = getattr(self, "is_wideband", False)

    @property
    def resids_init(self):
        """The pre-fit residuals (fitter.py:214 computes them at construction; here on first
        use, from the initial model)."""
        if self._resids_init is None:
            self._resids_init = self.make_resids(self.model_init)
        return self._resids_init

    @resids_init.setter
    def resids_init(self, r):
        self._resids_init = r

    @classmethod
    def auto(cls, toas, model, downhill=True, track_mode=None, residuals=None, **kwargs):
        """fitter.py:252 Fitter.auto (narrowband only)."""
        if model.has_correlated_errors:
            return (DownhillGLSFitter if downhill else GLSFitter)(toas, model, track_mode=track_mode)
        return (DownhillWLSFitter if downhill else WLSFitter)(toas, model, track_mode=track_mode)

    def make_resids(self, model):
        from .residuals import Residuals
        return Residuals(self.toas, model, track_mode=self.track_mode)

    def update_resids(self):
        self.resids = self.make_resids(self.model)

    def reset_model(self):
        """fitter.py:557: back to the initial model."""
        self.model = copy.deepcopy(self.model_init)
        self.update_resids()
        self.fitresult = []

    def get_designmatrix(self):
        return self.model.designmatrix(self.toas)

    def _run(self, mode, plain=True, threshold=None, style=None, noise=True, fac_style=None, **kw):
        from .engine import resident
        from .residuals import Residuals
        wideband = getattr(self, "is_wideband", False)
        # the resident upload of these TOAs and this model structure (engine.resident): a
        # refit, the next Downhill fit or a Residuals of the result re-binds one table
        s, lay = resident(self.model, self.toas, tag="wb" if wideband else None, track_mode=self.track_mode,
                          use_gls_basis=mode == "gls")
        bf = BatchFit([(self.model, self.toas)], mode=mode, session=s, layouts=[lay], threshold=threshold,
                      degeneracy_style=style, track_mode=self.track_mode, wideband=wideband, want_fac=True,
                      fac_style=fac_style)
        self.resids = None
        try:
            res = bf.fit_plain(**kw)[0] if plain else bf.fit_downhill(**kw)[0]
            # the final residuals are already on the device (the fit's last evaluation):
            # take them from the fit's own session instead of re-uploading (a WLS fit of a
            # correlated-noise model has no noise basis there, so its GLS chi2 is computed anew)
            if not wideband and (mode == "gls" or not self.model.has_correlated_errors):
                self.resids = Residuals._from_batch(self.toas, self.model, bf, 0, res.chi2, self.track_mode)
        finally:
            bf.close()
        self.fitresult = res
        self._set_outputs(res)
        if self.resids is None:
            self.update_resids()
        if mode == "gls" and noise and not wideband:
            self.resids.noise_resids = res.noise_resids
            self.resids.norm = res.fac  # fitter.py:2268-2282 sets resids.norm beside noise_resids
        if not plain:
            self.current_state = FitState(self, self.model, self.resids, res)
        return res

    def _set_outputs(self, res):
        """fitter.py:2231-2252 / :1076-1085: errors, the labelled covariance and correlation
        matrices of the fitted columns, and the step's normalisation ``fac``."""
        self.errors = res.errors
        self.parameter_covariance_matrix = CovarianceMatrix(res.cov, res.labels)
        self.parameter_correlation_matrix = self.parameter_covariance_matrix.to_correlation_matrix()
        self.converged = res.converged
        if not isinstance(self, DownhillFitter):  # DownhillFitter.fac is current_state.fac
            self.fac = res.fac

    # -- the reference Fitter's reporting API (fitter.py:348-620, :807-890) ------------
    def _get_corr_cov_matrix(self, matrix_type, with_phase, pretty_print, prec, usecolor):
        if not hasattr(self, f"parameter_{matrix_type}_matrix"):
            raise AttributeError(f"You must run .fit_toas() before accessing the {matrix_type} matrix")
        cm = getattr(self, f"parameter_{matrix_type}_matrix")
        if not pretty_print:
            return cm.prettyprint(prec=prec, offset=with_phase)
        print(cm.prettyprint(prec=prec, offset=with_phase, usecolor=usecolor))

    def get_parameter_covariance_matrix(self, with_phase=False, pretty_print=False, prec=3):
        """fitter.py:592."""
        return self._get_corr_cov_matrix("covariance", with_phase, pretty_print, prec, False)

    def get_parameter_correlation_matrix(self, with_phase=False, pretty_print=False, prec=3, usecolor=True):
        """fitter.py:605."""
        return self._get_corr_cov_matrix("correlation", with_phase, pretty_print, prec, usecolor)

    @property
    def covariance_matrix(self):
        warnings.warn("This parameter is deprecated. Use `parameter_covariance_matrix` instead of "
                      "`covariance_matrix`", DeprecationWarning)
        return self.parameter_covariance_matrix

    def get_params_dict(self, which="free", kind="value"):
        """fitter.py:807 (values, or uncertainties with kind="uncertainty")."""
        names = self.model.free_params if which == "free" else self.model.params
        if kind == "uncertainty":
            return {n: self.model[n].uncertainty for n in names}
        return self.model.get_params_dict(which=which)

    def set_param_uncertainties(self, fitp):
        """fitter.py:874."""
        for k, v in fitp.items():
            self.model[k].uncertainty = v

    def get_summary(self, nodmx=False):
        """fitter.py:348-472: fit quality and a prefit/postfit parameter table.  The layout
        (header lines, column widths, the uncertainties package's shorthand ``value(unc)``
        for fitted parameters) is the reference's; angles print as sexagesimal strings and
        the derived-parameter block (derived_quantities.py, out of scope) is omitted."""
        from .summary import fitter_summary
        return fitter_summary(self, nodmx=nodmx)

    def print_summary(self):
        """fitter.py:502."""
        print(self.get_summary())

    def update_model(self, chi2=None):
        """fitter.py:530-555: START/FINISH/NTOA (and EPHEM/CLOCK when the TOAs carry them),
        DMDATA; after a fit CHI2, CHI2R = chi2/dof and TRES = the weighted rms (us)."""
        from .parameter import LD, make_param
        m = self.model

        def par(name):
            if name not in m:
                m.add_param(make_param(name))
            return m[name]

        mj = self.toas.get_mjds()
        par("START").value = LD(np.min(mj))
        par("FINISH").value = LD(np.max(mj))
        par("NTOA").value = int(self.toas.ntoas)
        if getattr(self.toas, "ephem", None):
            par("EPHEM").value = self.toas.ephem
        if getattr(self.toas, "clock", None):
            par("CLOCK").value = self.toas.clock
        par("DMDATA").value = hasattr(self.resids, "dm")
        if chi2 is not None:
            par("CHI2").value = float(chi2)
            par("CHI2R").value = float(chi2) / self.resids.dof
            rw = self.resids.rms_weighted()
            if isinstance(rw, dict):  # wideband: TRES (us) and DMRES (pc/cm^3)
                par("TRES").value = float(rw["toa"])
                par("DMRES").value = float(rw["dm"])
            else:
                par("TRES").value = float(rw)

    def set_params(self, d):
        for k, v in d.items():
            self.model[k].value = v


class WLSFitter(Fitter):
    def __init__(self, toas, model, track_mode=None, residuals=None):
        super().__init__(toas, model, track_mode, residuals)
        self.method = "weighted_least_square"  # fitter.py:1963

    def fit_toas(self, maxiter=1, threshold=None, debug=False):
        if self.model.has_correlated_errors:
            pass  # the reference WLSFitter ignores correlated noise
        res = self._run("wls", plain=True, maxiter=maxiter, threshold=threshold, style="wls")
        self.update_model(res.chi2)
        return res.chi2


class GLSFitter(Fitter):
    def __init__(self, toas, model, track_mode=None, residuals=None):
        super().__init__(toas, model, track_mode, residuals)
        self.method = "generalized_least_square"  # fitter.py:2102

    def fit_toas(self, maxiter=1, threshold=0, full_cov=False, debug=False):
        """fitter.py:2104.  full_cov=True: the reference forms the dense N x N covariance
        C = N + U Phi U^T, Cholesky-factors it and solves M^T C^-1 M with the timing columns
        only (fitter.py:2180-2184).  By the Woodbury identity that system's solution and
        inverse are exactly the timing block of the rank-reduced system the device solves
        (the reference asserts the two agree, tests/test_gls_fitter.py:85-90), so both
        settings run the same device path; as in the reference, full_cov=True computes no
        noise realisations (fitter.py:2268)."""
        self.full_cov = full_cov
        res = self._run("gls", plain=True, maxiter=maxiter, threshold=threshold, style="gls",
                        noise=not full_cov, fac_style="timing" if full_cov else None)
        self.update_model(res.chi2)
        return res.chi2


class WidebandTOAFitter(Fitter):
    """fitter.py:2292-2637: a GLS fit of TOAs and their wideband DM measurements.  The design
    matrix is [M_toa | F; M_dm | 0] (the DM derivatives of every free parameter, zero
    noise-basis columns), the residuals [TOA residuals; pp_dm - DM] with the scaled TOA and
    DM errors.  On the device the DM rows only touch the DM-type columns and the residual of
    the normal equations (k_wb_gram, PINT_OPT_WBFIT); the rest is the GLS step.  Needs the
    compact DMX layout (>= 8 free DMX bins, no TOA in two bins, no ECORR)."""

    def __init__(self, fit_data, model, fit_data_names=["toa", "dm"], track_mode=None, additional_args={}):
        toas = fit_data[0] if isinstance(fit_data, (list, tuple)) else fit_data
        if not hasattr(toas, "is_wideband"):
            raise ValueError(f"The first data set should be a TOAs object but is {toas}.")
        if len(fit_data_names) == 0:
            raise ValueError("Please specify the fit data.")
        super().__init__(toas, model, track_mode=track_mode)
        self.fit_data_names = list(fit_data_names)
        self.additional_args = dict(additional_args)
        self.is_wideband = True
        self.method = "General_Data_Fitter"
        self.update_resids()
        self.resids_init = self.resids

    def make_resids(self, model):
        from .residuals import WidebandTOAResiduals
        ta = dict(self.additional_args.get("toa", {}))
        if self.track_mode is not None:
            ta["track_mode"] = self.track_mode
        return WidebandTOAResiduals(self.toas, model, toa_resid_args=ta, dm_resid_args=self.additional_args.get("dm", {}))

    def fit_toas(self, maxiter=1, threshold=0, full_cov=False, debug=False):
        """Returns the last step's linearised chi2 (newres^T C^-1 newres + xhat^T phi^-1 xhat,
        fitter.py:2546-2552); full_cov=True solves the same system (Woodbury identity)."""
        self.model.validate()
        bf = BatchFit([(self.model, self.toas)], mode="gls", threshold=threshold, degeneracy_style="gls",
                      track_mode=self.track_mode, wideband=True, want_fac=True)
        try:
            res = bf.fit_plain(maxiter=maxiter)[0]
            chi2 = float(bf.last_chi2_lin[0])
        finally:
            bf.close()
        self.fitresult = res
        self._set_outputs(res)
        self.update_resids()
        self.update_model(chi2)
        return chi2


class DownhillFitter(Fitter):
    mode = "wls"

    def __init__(self, toas, model, track_mode=None, residuals=None):
        super().__init__(toas, model, track_mode, residuals)
        self.method = "downhill_checked"  # fitter.py:997

    @property
    def fac(self):
        """fitter.py:1207: the normalisation of the best state's step."""
        return self.current_state.fac

    def fit_toas(self, maxiter=20, noise_fit_niter=2, required_chi2_decrease=1e-2, max_chi2_increase=1e-2,
                 min_lambda=1e-3, noisefit_method="Newton-CG", compute_noise_uncertainties=True, debug=False,
                 threshold=None, **kw):
        """fitter.py:1107-1204.  No free noise parameters: one downhill fit, with
        required_chi2_decrease passed as both max_chi2_increase and min_lambda (a reference
        quirk, fitter.py:1168-1175).  Free EFAC/EQUAD/ECORR/red-noise parameters: timing
        fits alternate with noise-likelihood maximisations (pint_amd.noisefit.fit_noise, on
        the device) noise_fit_niter times, then a final timing fit; the last noise fit also
        sets the noise uncertainties when compute_noise_uncertainties.  Exceptions of the
        timing fits (StepProblem, MaxiterReached) propagate as in the reference."""
        from .noisefit import fit_noise
        free_noise = self._get_free_noise_params()
        if not free_noise:
            return self._fit_toas(maxiter, required_chi2_decrease, required_chi2_decrease, required_chi2_decrease,
                                  threshold)
        for ii in range(noise_fit_niter):
            self._fit_toas(maxiter, required_chi2_decrease, max_chi2_increase, min_lambda, threshold)
            if ii == noise_fit_niter - 1 and compute_noise_uncertainties:
                values, errors = fit_noise(self.toas, self.model, noisefit_method, uncertainty=True)
                self._update_noise_params(values, errors)
            else:
                values = fit_noise(self.toas, self.model, noisefit_method, uncertainty=False)
                self._update_noise_params(values)
        return self._fit_toas(maxiter, required_chi2_decrease, max_chi2_increase, min_lambda, threshold)

    def _get_free_noise_params(self):
        """fitter.py:1210."""
        from .noisefit import free_noise_params
        return free_noise_params(self.model)

    def _update_noise_params(self, values, errors=None):
        """fitter.py:1218."""
        for k, fp in enumerate(self._get_free_noise_params()):
            self.model[fp].value = float(values[k])
            if errors is not None:
                self.model[fp].uncertainty_value = float(errors[k])

    def _fit_toas(self, maxiter, required_chi2_decrease, max_chi2_increase, min_lambda, threshold=None):
        """fitter.py:1023-1105 (threshold: WLSState None -> 1e-14 max(N, P), GLSState
        fitter.py:1554 default 0)."""
        if threshold is None and self.mode == "gls":
            threshold = 0.0
        res = self._run(self.mode, plain=False, maxiter=maxiter, required_chi2_decrease=required_chi2_decrease,
                        max_chi2_increase=max_chi2_increase, min_lambda=min_lambda,
                        threshold=threshold, style="wls" if self.mode == "wls" else "glsstate",
                        fac_style="wbstate" if getattr(self, "is_wideband", False) else None)
        self.update_model(res.chi2)
        if res.status == "StepProblem":
            raise StepProblem("Unable to improve chi2 even with very small steps")
        if not res.converged:
            raise MaxiterReached(f"Convergence not detected after {maxiter} steps.")
        return self.converged


class WidebandDownhillFitter(DownhillFitter):
    """fitter.py:1812-1895: the downhill line search (DownhillFitter._fit_toas) with the
    wideband step (WidebandState: the GLS step over [TOA rows; DM rows], fitter.py:1612-1810)
    and the wideband chi2 (WidebandTOAResiduals); on the device the step is the GLS step with
    k_wb_gram and every trial's chi2 adds the DM chi2 (BatchFit(wideband=True))."""
    mode = "gls"

    def __init__(self, toas, model, track_mode=None, residuals=None, add_args=None):
        self.add_args = {} if add_args is None else add_args
        self.is_wideband = True
        self.full_cov = False
        self.threshold = 0
        super().__init__(toas, model, track_mode, residuals)
        self.method = "downhill_wideband"

    def make_resids(self, model):
        from .residuals import WidebandTOAResiduals
        return WidebandTOAResiduals(self.toas, model, toa_resid_args=self.add_args.get("toa", {}),
                                    dm_resid_args=self.add_args.get("dm", {}))

    def fit_toas(self, maxiter=10, threshold=1e-14, full_cov=False, debug=False, **kwargs):
        """threshold: WidebandState's SVD cut (the device solves by Cholesky and takes the SVD
        path only for degenerate normal equations); full_cov solves the same system."""
        self.threshold = threshold
        self.full_cov = full_cov
        return super().fit_toas(maxiter=maxiter, debug=debug, threshold=threshold, **kwargs)


class DownhillWLSFitter(DownhillFitter):
    mode = "wls"

    def __init__(self, toas, model, track_mode=None, residuals=None):
        if model.has_correlated_errors:
            raise CorrelatedErrors(model)
        super().__init__(toas, model, track_mode, residuals)
        self.method = "downhill_wls"  # fitter.py:1392


class DownhillGLSFitter(DownhillFitter):
    mode = "gls"

    def __init__(self, toas, model, track_mode=None, residuals=None):
        super().__init__(toas, model, track_mode, residuals)
        self.method = "downhill_gls"  # fitter.py:1545
