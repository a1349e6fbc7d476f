"""grid_chisq, grid_chisq_derived, tuple_chisq and tuple_chisq_derived (reference
gridutils.py:166-966) on the GPU.

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
import os
from typing import List, Sequence

import numpy as np

from .fitter import (BatchFit, DownhillFitter, GLSFitter, DownhillGLSFitter, WLSFitter, model_key)
from .parameter import LD


GRID_BATCH_BYTES = 24e9   # device bytes one batch of grid points may take
GRID_MAX_POINTS = None    # optional cap on points per batch
# Concurrent pipelines per rank: a batch of points is split into GRID_PIPES contiguous blocks,
# each fitted on a Session of its own (its own streams and buffers, the same uploaded pulsar)
# with all launches enqueued before any is waited on -- a grid point's kernels are short and
# latency-bound, and the second block's run in the first one's gaps.  A rank's points stay
# on one session unless every block gets GRID_PIPE_MIN points: the host enqueues each block's
# launches, and below that the second enqueue cost more than the overlap gave (measured on
# the 256 x 256 NGC6440E grid: 65,536 points 0.93 -> 0.89 ms with two sessions; blocks of
# 16,384 and 8,192 points 0.39 -> 0.44 and 0.31 -> 0.37 ms).  (PINT_GRID_PIPES overrides.)
GRID_PIPES = int(os.environ.get("PINT_GRID_PIPES", "2"))
GRID_PIPE_MIN = 16384


def _fit_kind(ftr):
    gls = isinstance(ftr, (GLSFitter, DownhillGLSFitter))
    down = isinstance(ftr, DownhillFitter)
    return ("gls" if gls else "wls"), down


def grid_points(parvalues):
    out = np.meshgrid(*[np.asarray(v, dtype=np.longdouble) for v in parvalues])
    return out, [o.flatten() for o in out]


def meshgrid_axes(parvalues):
    """The flattened np.meshgrid(*parvalues) (indexing 'xy') as axes: for parameter j, its
    axis values and (stride, size) such that flat point k takes values[(k // stride) % size]
    -- what pint_set_grid forms on the device, without the flattened meshgrid."""
    axes = [np.asarray(v, dtype=np.longdouble).reshape(-1) for v in parvalues]
    n = [a.size for a in axes]
    shape = list(n)
    if len(n) >= 2:  # 'xy': the first two axes swap
        shape[0], shape[1] = n[1], n[0]
    ax_of = list(range(len(n)))
    if len(n) >= 2:
        ax_of[0], ax_of[1] = 1, 0
    out = []
    for j, a in enumerate(axes):
        ax = ax_of[j]
        stride = int(np.prod(shape[ax + 1:], dtype=np.int64)) if ax + 1 < len(shape) else 1
        out.append((a, stride, shape[ax]))
    return out, int(np.prod(shape, dtype=np.int64))


def meshgrid_shape(parvalues):
    """np.meshgrid(*parvalues)[0].shape (indexing 'xy': the first two axes swap), from the
    axis lengths alone."""
    n = [np.atleast_1d(v).size for v in parvalues]
    if len(n) >= 2:
        n[0], n[1] = n[1], n[0]
    return tuple(n)


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


def shard_range(npts: int, rank: int, world: int):
    """Contiguous block [lo, hi) of the flattened meshgrid owned by `rank`."""
    per = (npts + world - 1) // world
    return per, rank * per, min(npts, (rank + 1) * per)


def gather_blocks(local: np.ndarray, per: int, npts: int, dist) -> np.ndarray:
    """All-gather every rank's chi2 block (NaN-padded to `per`) -> the full flat array.
    Over RCCL when the process group is nccl, gloo on CPU."""
    from . import pta
    if dist is None or (dist.get_world_size() == 1 and not pta.FORCE_COLLECTIVE):
        return local
    import torch
    world = dist.get_world_size()
    buf = torch.full((per,), float("nan"), dtype=torch.float64)
    buf[: len(local)] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64))
    if dist.get_backend() == "nccl":  # this rank's GPU (LOCAL_RANK), not whatever device is current
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        buf = buf.to(dev)
    gl = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(gl, buf)
    return torch.cat([g.cpu() for g in gl]).numpy()[:npts]


# The last grid's Session and uploaded pulsar stay resident (like the TOAs of a serving
# process): another grid over the same TOAs and model structure reuses the upload.  The
# key holds everything the layout depends on -- the TOA object, and every parameter's
# name, value and frozen flag (noise parameters set the basis weights) -- so any change
# re-uploads.
_GRID = {}
# (rank, world) whose contiguous block alone a grid call fits, without a process group: the
# bench's per-rank prediction of an N-rank grid on one GPU (None: the real rank and world)
_EMULATE_SHARD = None


def _grid_session(model, parnames, toas, gls, npipe=1):
    """The resident Sessions (npipe of them, each with the pulsar uploaded) and their layouts
    for grids of `model` with `parnames` frozen (a copy of the model is made and frozen only
    when a new upload is needed: the copy cost ~0.7 ms per grid)."""
    from .engine import Session, build_layout
    key = (id(toas), toas.ntoas, gls, model_key(model, freeze=tuple(parnames)))
    cur = _GRID.get("cur")
    if cur is None or cur[0] != key or cur[3] is not toas:
        _drop_grid_session()
        base = copy.deepcopy(model)
        for p in parnames:
            base[p].frozen = True
        cur = _GRID["cur"] = (key, [], base, toas)
    pipes, base = cur[1], cur[2]
    while len(pipes) < npipe:
        s = Session()
        # a grid point reports its post-fit chi2, which is second order in a step error along
        # the weak directions: the solves' iterative refinement (PINT_OPT_REFINE) buys nothing
        s.set_refine(False)
        s.set_timing_mask(0)  # no timing events in a grid's steps (bench.grid_leg turns them on)
        try:
            lay = s.add(build_layout(base, toas, use_gls_basis=gls))
        except Exception:
            s.close()
            raise
        pipes.append((s, lay))
    return pipes[:npipe]


def _drop_grid_session():
    cur = _GRID.pop("cur", None)
    if cur is not None:
        for s, _ in cur[1]:
            s.close()


def _fit_block(s, lay, grid, mode, down, fitargs, want_tables):
    """Fit one batch of grid points of the uploaded pulsar `lay` (grid: (base table, variables,
    npts, k0), the points' tables formed on the device), every point its own instance.
    Returns (chi2, final tables or None); a point that cannot be evaluated is NaN
    (gridutils.py:101-106), and so is every point of a batch in which no point can be."""
    from .fitter import InvalidModelParameters
    base, variables, npts, k0 = grid
    if not down:
        got = _fit_block_enqueued(s, lay, grid, mode, fitargs, want_tables)
        if got is not None:
            return got
    bf = BatchFit(None, mode=mode, session=s, grid=(lay, base, variables, npts, k0))
    try:
        if down:
            rq = fitargs.get("required_chi2_decrease", 1e-2)
            res = bf.fit_downhill(maxiter=fitargs.get("maxiter", 10), required_chi2_decrease=rq,
                                  max_chi2_increase=rq, min_lambda=rq, outputs=False)
            # gridutils.py:89-106: NaN on MaxiterReached, chi2 kept on StepProblem
            chi2 = np.where(res.maxiter_reached, np.nan, res.chi2)
        else:
            res = bf.fit_plain(maxiter=fitargs.get("maxiter", 1), outputs=False)
            chi2 = res.chi2
    except InvalidModelParameters:
        return np.full(npts, np.nan), (np.full((npts, lay.tstride), np.nan) if want_tables else None)
    ft = bf.final_tables_flat().reshape(npts, lay.tstride) if want_tables else None
    return chi2, ft


def _fit_block_enqueued(s, lay, grid, mode, fitargs, want_tables):
    """_fit_block's plain fit (maxiter steps, then the chi2) with every launch enqueued and
    one synchronisation at the end (lazy Session): the synchronous form waited on the
    device after each of its five calls (~40 us of idle device each at 65,536 points).
    Returns None -- and the caller refits the block synchronously, which handles them -- if
    any point raised a status (an invalid point, a degenerate normal matrix)."""
    return _fit_block_finish(s, lay, _fit_block_start(s, lay, grid, mode, fitargs), grid[2], want_tables)


def _fit_block_start(s, lay, grid, mode, fitargs):
    """The launches of _fit_block_enqueued, enqueued (lazy Session, nothing waited on);
    returns what _fit_block_finish takes, or None after a status raised while enqueueing."""
    from . import _lib as L
    base, variables, npts, k0 = grid
    s.set_lazy(True)
    try:
        # (lazy from the binding on: pint_set_grid then leaves its upload to the stream)
        bf = BatchFit(None, mode=mode, session=s, grid=(lay, base, variables, npts, k0))
        for _ in range(fitargs.get("maxiter", 1)):
            s.eval(want_M=s.FIT)
            s.fit_step(1 if bf.gls else 0)
            s.apply_step_uniform(1.0)
        s.eval(want_M=False)
        return bf, bf._chi2_enqueue()
    except L.PintError as e:
        s.set_lazy(False)
        if e.code not in BatchFit.EVAL_ERRORS + (L.PINT_E_NOT_PD,):
            raise
        return None


def _fit_block_finish(s, lay, started, npts, want_tables):
    """Wait for a block _fit_block_start enqueued: (chi2, final tables or None), or None
    if any point raised a status."""
    from . import _lib as L
    if started is None:
        return None
    bf, get = started
    try:
        s.check()
        chi2 = np.array(get()[0], dtype=np.float64)
    except L.PintError as e:
        if e.code not in BatchFit.EVAL_ERRORS + (L.PINT_E_NOT_PD,):
            raise
        return None
    finally:
        s.set_lazy(False)
    ft = bf.final_tables_flat().reshape(npts, lay.tstride) if want_tables else None
    return chi2, ft


def point_tables(lay, base_table, parnames, flat, c0, c1):
    """Parameter tables of grid points c0..c1 (flattened meshgrid order): the base model's
    table with each grid parameter's dd pair replaced."""
    tabs = np.tile(base_table, (c1 - c0, 1))
    for p, vals in zip(parnames, flat):
        v = np.asarray(vals[c0:c1], dtype=np.longdouble)
        h = v.astype(np.float64)
        l = (v - h.astype(np.longdouble)).astype(np.float64)
        o = lay.offsets[p]
        tabs[:, o] = h
        tabs[:, o + 1] = l
    return tabs


def _as_ld(v):
    """A grid coordinate as longdouble: plain numbers, numpy arrays, or anything carrying a
    `.value` in the parameter's own unit (the reference passes astropy Quantities)."""
    return np.asarray(getattr(v, "value", v), dtype=np.longdouble)


def _chisq_flat(ftr, parnames: Sequence[str], flat: Sequence[np.ndarray],
                extraparnames: Sequence[str], fitargs, axes=None):
    """Fit every point of `flat` (one longdouble array of values per parameter in
    `parnames`, all of one length) with `parnames` frozen; returns the flat chi2 array and a
    dict of flat extra-parameter arrays, every rank holding all points.  The shared body of
    the four grid entry points (gridutils.py:166/:392/:588/:773, parallel path: a cold
    start from the input fitter's model at every point, gridutils.py:72).  axes: instead of
    `flat`, (meshgrid_axes output, npts) -- the points formed on the device from the axes."""
    from .engine import pack_table
    mode, down = _fit_kind(ftr)
    if axes is not None:
        axes, npts = axes
    else:
        npts = int(flat[0].size) if len(flat) else 0
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    if _EMULATE_SHARD is not None:  # (bench.py's predicted_strong: one rank's block of an N-rank run, alone)
        rank, world = _EMULATE_SHARD
        dist = None
    per, lo, hi = shard_range(npts, rank, world)
    chi2 = np.full(hi - lo, np.nan)
    extra = {e: np.full(hi - lo, np.nan) for e in extraparnames}
    if hi > lo:
        npipe = max(1, min(GRID_PIPES, (hi - lo) // GRID_PIPE_MIN)) if not down else 1
        pipes = _grid_session(ftr.model, parnames, ftr.toas, mode == "gls", npipe)
        lay = pipes[0][1]
        want = bool(extraparnames)
        try:
            t0 = pack_table(lay, ftr.model)  # (the frozen flags do not enter the table)
            # points per batch: ~24 GB of per-instance device buffers (eval rows, design matrix,
            # Gram partials) per batch and pipeline keeps any grid within HBM
            per_pt = 8.0 * (lay.n * (lay.K + 12) + 64 * (lay.K + 2) ** 2)
            chunk = int(max(1, min(hi - lo, GRID_BATCH_BYTES // per_pt * npipe, GRID_MAX_POINTS or hi - lo)))

            def block(c0, c1):  # grid points [c0, c1) as _fit_block's grid argument
                if axes is not None:   # meshgrid axes: point k of the block is flat point c0 + k
                    var = [(p, a, st, sz) for p, (a, st, sz) in zip(parnames, axes)]
                    return (t0, var, c1 - c0, c0)
                var = [(p, np.asarray(v[c0:c1], dtype=np.longdouble), 1, c1 - c0) for p, v in zip(parnames, flat)]
                return (t0, var, c1 - c0, 0)   # every point's own values

            def store(c0, c1, c2, ft):
                chi2[c0 - lo:c1 - lo] = c2
                for e in extraparnames:
                    o = lay.offsets[e]
                    extra[e][c0 - lo:c1 - lo] = (ft[:, o].astype(np.longdouble)
                                                 + ft[:, o + 1].astype(np.longdouble)).astype(np.float64)

            for c0 in range(lo, hi, chunk):
                c1 = min(hi, c0 + chunk)
                if npipe == 1:
                    store(c0, c1, *_fit_block(pipes[0][0], lay, block(c0, c1), mode, down, fitargs, want))
                    continue
                # the chunk's npipe contiguous blocks, every block's launches enqueued on its
                # own session before any is waited on
                cuts = [c0 + (c1 - c0) * k // npipe for k in range(npipe + 1)]
                subs = [(cuts[k], cuts[k + 1], block(cuts[k], cuts[k + 1])) for k in range(npipe)]
                started = [_fit_block_start(ps, pl, g, mode, fitargs) for (ps, pl), (_, _, g) in zip(pipes, subs)]
                for (ps, pl), (b0, b1, g), st in zip(pipes, subs, started):
                    got = _fit_block_finish(ps, pl, st, b1 - b0, want)
                    if got is None:  # a status: that block refitted synchronously (_fit_block)
                        got = _fit_block(ps, pl, g, mode, down, fitargs, want)
                    store(b0, b1, *got)
        except Exception:
            _drop_grid_session()
            raise
    # extras are the point's parameter values after its fit, also for a MaxiterReached point
    # (gridutils.py:107-110 reads them outside the try); a point taken out of the batch as
    # invalid has none (NaN, final_tables_flat)
    if _EMULATE_SHARD is not None:  # the block in place, NaN elsewhere
        def place(v):
            out = np.full(npts, np.nan)
            out[lo:hi] = v
            return out
        return place(chi2), {e: place(extra[e]) for e in extraparnames}
    chi2_all = gather_blocks(chi2, per, npts, dist)
    extra_all = {e: gather_blocks(extra[e], per, npts, dist) for e in extraparnames}
    return chi2_all, extra_all


def grid_chisq(ftr, parnames: Sequence[str], parvalues: Sequence, extraparnames: List[str] = [],
               executor=None, ncpu=None, chunksize=1, printprogress=False, **fitargs):
    """chi2 over the meshgrid of `parvalues` with `parnames` frozen (gridutils.py:166).
    Returns (chi2 array of meshgrid shape, dict of meshgrid-shaped extra parameter arrays).
    `executor`, `ncpu`, `chunksize` are accepted for API compatibility: the points run as one
    GPU batch per rank instead of a process pool.  With torch.distributed initialised, rank
    r fits the r-th contiguous block of the flattened meshgrid and the blocks are
    all-gathered, so every rank returns the whole grid."""
    shape = meshgrid_shape(parvalues)
    chi2, extra = _chisq_flat(ftr, parnames, None, extraparnames, fitargs, axes=meshgrid_axes(parvalues))
    return chi2.reshape(shape), {e: v.reshape(shape) for e, v in extra.items()}


def grid_chisq_derived(ftr, parnames: Sequence[str], parfuncs: Sequence, gridvalues: Sequence,
                       extraparnames: List[str] = [], executor=None, ncpu=None, chunksize=1,
                       printprogress=False, **fitargs):
    """chi2 over the meshgrid of `gridvalues`, each point's fitted parameters `parnames` set to
    `parfuncs[j](*grid)` (gridutils.py:392-585): e.g. a grid in (F0, tau) fitting F0 and
    F1 = -F0 / 2 tau.  Returns (chi2 of meshgrid shape, [parameter value arrays of meshgrid
    shape, one per parfunc], dict of meshgrid-shaped extras).  The functions see longdouble
    meshgrids; the extras follow the reference's parallel path (one array entry per point --
    its serial path keeps only the last point's value, gridutils.py:580-581)."""
    grid = np.meshgrid(*[_as_ld(v) for v in gridvalues])
    shape = grid[0].shape
    # writable arrays of meshgrid shape (a parfunc returning a scalar broadcasts to a copy,
    # not to a read-only stride-0 view)
    out = [np.array(np.broadcast_to(np.asarray(f(*grid)), shape)) for f in parfuncs]
    flat = [_as_ld(o).reshape(-1) for o in out]
    chi2, extra = _chisq_flat(ftr, parnames, flat, extraparnames, fitargs)
    return chi2.reshape(shape), out, {e: v.reshape(shape) for e, v in extra.items()}


def tuple_chisq(ftr, parnames: Sequence[str], parvalues: Sequence, extraparnames: List[str] = [],
                executor=None, ncpu=None, chunksize=1, printprogress=False, **fitargs):
    """chi2 at each tuple of `parvalues` (one value per name of `parnames`, any set of points:
    gridutils.py:588-770).  Returns (chi2 of length len(parvalues), dict of extra-parameter
    arrays of that length).  Multi-GPU: the list is split into contiguous blocks, one per
    rank, exactly like the flattened meshgrid of grid_chisq."""
    flat = [_as_ld([pv[j] for pv in parvalues]).reshape(-1) for j in range(len(parnames))]
    return _chisq_flat(ftr, parnames, flat, extraparnames, fitargs)


def tuple_chisq_derived(ftr, parnames: Sequence[str], parfuncs: Sequence, parvalues: Sequence,
                        extraparnames: List[str] = [], executor=None, ncpu=None, chunksize=1,
                        printprogress=False, **fitargs):
    """chi2 at each tuple of `parvalues`, the fitted parameters `parnames` set to
    `[f(*tuple) for f in parfuncs]` (gridutils.py:773-966).  Returns (chi2, the list of
    per-point parameter value lists, dict of extras)."""
    out = [[f(*pv) for f in parfuncs] for pv in parvalues]
    flat = [_as_ld([o[j] for o in out]).reshape(-1) for j in range(len(parnames))]
    chi2, extra = _chisq_flat(ftr, parnames, flat, extraparnames, fitargs)
    return chi2, out, extra


def best_point(chi2, parnames: Sequence[str], parvalues: Sequence):
    """The grid's best-fit point: (meshgrid index, {name: value}, chi2).  Every rank holds the
    all-gathered grid, so the reduction is a host argmin (NaN points never win)."""
    c = np.asarray(chi2)
    if np.all(np.isnan(c)):
        raise ValueError("no grid point has a chi2")
    k = np.unravel_index(int(np.nanargmin(c)), c.shape)
    out, _ = grid_points(parvalues)
    return k, {p: out[j][k] for j, p in enumerate(parnames)}, float(c[k])
