"""grid_chisq (reference gridutils.py:166-389) on the GPU.

Every grid point is one parameter-table instance; all points of a rank are fitted by one
batched launch sequence (BatchFit).  Semantics follow the reference's *parallel* path
(gridutils.py:72 deep copy per point = cold start from the input fitter's model); the
serial ncpu=1 path of the reference warm-starts and can differ for non-converging points
(SURVEY.md §8(e)).  Multi-GPU: when torch.distributed is initialised, the flattened
meshgrid (np.ndindex order, gridutils.py:331/:366) is split into contiguous blocks, one per
rank, and the chi2 blocks are all-gathered over RCCL -- the only collective.
"""
from __future__ import annotations

import copy
from typing import List, Sequence

import numpy as np

from .fitter import (BatchFit, DownhillFitter, GLSFitter, DownhillGLSFitter, WLSFitter)
from .parameter import LD


def _fit_kind(ftr):
    gls = isinstance(ftr, (GLSFitter, DownhillGLSFitter))
    down = isinstance(ftr, DownhillFitter)
    return ("gls" if gls else "wls"), down


def grid_points(parvalues):
    out = np.meshgrid(*[np.asarray(v, dtype=np.longdouble) for v in parvalues])
    return out, [o.flatten() for o in out]


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


def grid_chisq(ftr, parnames: Sequence[str], parvalues: Sequence, extraparnames: List[str] = [],
               executor=None, ncpu=None, chunksize=1, printprogress=False, **fitargs):
    """chi2 over the meshgrid of `parvalues` with `parnames` frozen (gridutils.py:166).
    Returns (chi2 array of meshgrid shape, dict of extra parameter arrays)."""
    mode, down = _fit_kind(ftr)
    out, flat = grid_points(parvalues)
    shape = out[0].shape
    npts = flat[0].size
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    per = (npts + world - 1) // world
    lo, hi = rank * per, min(npts, (rank + 1) * per)
    base = copy.deepcopy(ftr.model)
    for p in parnames:
        base[p].frozen = True
    items = []
    for i in range(lo, hi):
        m = copy.deepcopy(base)
        for p, vals in zip(parnames, flat):
            m[p].value = LD(vals[i]) if (m[p].long_double or m[p].kind == "mjd") else float(vals[i])
        items.append((m, ftr.toas))
    chi2 = np.full(hi - lo, np.nan)
    extra = {e: np.full(hi - lo, np.nan) for e in extraparnames}
    if items:
        bf = BatchFit(items, mode=mode, layouts=_shared_layouts(items, mode))
        try:
            if down:
                kw = dict(maxiter=fitargs.get("maxiter", 10))
                rq = fitargs.get("required_chi2_decrease", 1e-2)
                res = bf.fit_downhill(required_chi2_decrease=rq, max_chi2_increase=rq, min_lambda=rq, **kw)
            else:
                res = bf.fit_plain(maxiter=fitargs.get("maxiter", 1))
        finally:
            bf.close()
        for k, r in enumerate(res):
            # gridutils.py:89-106: NaN on MaxiterReached, chi2 kept on StepProblem
            chi2[k] = np.nan if (down and r.status == "MaxiterReached") else r.chi2
            for e in extraparnames:
                extra[e][k] = float(items[k][0][e].value)
    if dist and world > 1:
        import torch
        buf = torch.full((per,), float("nan"), dtype=torch.float64)
        buf[: hi - lo] = torch.from_numpy(chi2)
        gathered = [torch.empty_like(buf) for _ in range(world)]
        dev_buf = buf.cuda() if torch.cuda.is_available() and dist.get_backend() == "nccl" else buf
        gl = [g.to(dev_buf.device) for g in gathered]
        dist.all_gather(gl, dev_buf)
        chi2_all = torch.cat([g.cpu() for g in gl]).numpy()[:npts]
    else:
        chi2_all = chi2
    extraout = {e: extra[e] for e in extraparnames}
    return chi2_all.reshape(shape), extraout


def _shared_layouts(items, mode):
    """All grid points share one uploaded pulsar (same TOAs and structure)."""
    from .engine import build_layout
    return None
