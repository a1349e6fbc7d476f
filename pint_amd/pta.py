"""A pulsar timing array's fits across the GPUs of a node.

The pulsars of a PTA are independent fits (each its own TimingModel + TOAs, the reference
fits them one after the other).  Here they are sharded over the ranks of a
torch.distributed group, one process per GPU:

* assignment: greedy longest-processing-time on the cost N K^2 + 8 N P of a fit (the
  Gram's 2 N K^2 flops and the design matrix's 8 N P bytes), so the
  ranks' batches finish together;
* each rank fits its pulsars as ONE batch (BatchFit: one launch sequence for all of them);
* the per-pulsar fit records (chi2, status, fitted values as double-double pairs, errors)
  are all-gathered -- over RCCL when the group's backend is nccl, gloo on CPU -- and every
  rank writes all of them into its models, so each rank ends with the whole fitted PTA.

That gather is the only collective; there is no data-path communication.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

import numpy as np

# Run the gathers through the process group even at world size 1 (tests: the RCCL branch
# executes on one GPU before a multi-GPU node ever sees it).
FORCE_COLLECTIVE = False

STATUS_CODES = {"ok": 0, "converged": 1, "MaxiterReached": 2, "StepProblem": 3, "InvalidModelParameters": 4}
STATUS_NAMES = {v: k for k, v in STATUS_CODES.items()}


def fit_cost(model, toas=None, n: Optional[int] = None) -> float:
    """Cost of one fit: N K^2 (Gram) + 8 N P (design matrix), K = P + 2 nred."""
    n = toas.ntoas if toas is not None else n
    P = len(model.free_params) + 1
    nred = model.red_noise_params()[2] if "PLRedNoise" in model.components else 0
    K = P + 2 * nred
    return float(n) * K * K + 8.0 * n * P


def lpt_shard(costs: Sequence[float], world: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment: items in decreasing cost, each to the
    least-loaded rank (lowest rank on ties).  Deterministic, so every rank computes the same
    assignment without communicating."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        out[r].append(i)
        load[r] += costs[i]
    for o in out:
        o.sort()
    return out


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


def gather_rows(local: np.ndarray, counts: Sequence[int], dist) -> np.ndarray:
    """All-gather each rank's (counts[r], W) float64 block; returns the rank-ordered
    concatenation (sum(counts), W) on every rank.  RCCL for an nccl group, gloo on CPU."""
    if dist is None or (dist.get_world_size() == 1 and not FORCE_COLLECTIVE):
        return local
    import torch
    W = local.shape[1]
    mx = max(max(counts), 1)
    buf = torch.full((mx, W), float("nan"), dtype=torch.float64)
    if len(local):
        buf[: len(local)] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64))
    if dist.get_backend() == "nccl":
        # this rank's own GPU (LOCAL_RANK), whatever device is current: a collective over
        # buffers that all landed on cuda:0 hangs or fails in RCCL
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        buf = buf.to(dev)
    gl = [torch.empty_like(buf) for _ in range(dist.get_world_size())]
    dist.all_gather(gl, buf)
    return np.concatenate([g.cpu().numpy()[:c] for g, c in zip(gl, counts)])


def _record_width(items) -> int:
    return 4 + 3 * max(len(m.free_params) for m, _ in items)


def _pack(i, model, res, width) -> np.ndarray:
    """[index, chi2, status, nfree, hi(nfree), lo(nfree), err(nfree)] padded with NaN."""
    from .engine import split_ld
    rec = np.full(width, np.nan)
    free = list(model.free_params)
    nf = len(free)
    rec[0], rec[1], rec[2], rec[3] = i, res.chi2, STATUS_CODES.get(res.status, 0), nf
    for j, p in enumerate(free):
        v = model[p].value
        rec[4 + j], rec[4 + nf + j] = split_ld(0.0 if v is None else v)
        e = model[p].uncertainty
        rec[4 + 2 * nf + j] = np.nan if e is None else e
    return rec


def _unpack(rec, model, res):
    from .parameter import LD
    free = list(model.free_params)
    nf = int(rec[3])
    res.chi2 = float(rec[1])
    res.status = STATUS_NAMES.get(int(rec[2]), "ok")
    res.converged = res.status in ("ok", "converged")
    if res.status == "InvalidModelParameters":
        return
    for j, p in enumerate(free[:nf]):
        par = model[p]
        v = LD(rec[4 + j]) + LD(rec[4 + nf + j])
        par.value = v if (par.long_double or par.kind == "mjd") else float(v)
        par.uncertainty = float(rec[4 + 2 * nf + j])
    res.errors = rec[4 + 2 * nf:4 + 3 * nf].copy()


def fit_pta(items: Sequence[tuple], mode: str = "gls", downhill: bool = False, maxiter: Optional[int] = None,
            dist=None, fit_fn: Optional[Callable] = None, **fitargs):
    """Fit every (model, toas) of a PTA, sharded over the ranks of `dist` (default: the
    initialised torch.distributed group, or one process).  Returns (results, shards): a
    FitResult per pulsar in input order (on every rank) and the rank -> pulsar assignment.
    Every model is updated in place on every rank.  The per-rank covariance matrices stay
    on the rank that fitted the pulsar (results[i].cov is None elsewhere).

    fit_fn(items, mode, downhill, maxiter, **fitargs) -> [FitResult] replaces the per-rank
    batched GPU fit (tests stub it to exercise the sharding and the gather on CPU)."""
    from .fitter import FitResult
    dist = dist if dist is not None else _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    items = list(items)
    shards = lpt_shard([fit_cost(m, t) for m, t in items], world)
    mine = shards[rank]
    fit_fn = fit_fn or _batch_fit
    local = fit_fn([items[i] for i in mine], mode, downhill, maxiter, **fitargs) if mine else []
    width = _record_width(items)
    recs = np.stack([_pack(i, items[i][0], r, width) for i, r in zip(mine, local)]) if mine \
        else np.zeros((0, width))
    allrec = gather_rows(recs, [len(s) for s in shards], dist)
    results = [FitResult() for _ in items]
    for i, r in zip(mine, local):
        results[i] = r
    for rec in allrec:
        i = int(rec[0])
        if i in mine:
            continue
        _unpack(rec, items[i][0], results[i])
    return results, shards


def _batch_fit(items, mode, downhill, maxiter, **fitargs):
    from .fitter import BatchFit
    bf = BatchFit(items, mode=mode)
    try:
        if downhill:
            rq = fitargs.get("required_chi2_decrease", 1e-2)
            return bf.fit_downhill(maxiter=maxiter or 10, required_chi2_decrease=rq, max_chi2_increase=rq,
                                   min_lambda=rq)
        return bf.fit_plain(maxiter=maxiter or 1)
    finally:
        bf.close()
