"""Multi-rank paths on CPU (gloo, world size 2): grid_chisq sharded over ranks end to end and
a PTA's pulsars sharded by LPT with the per-pulsar records all-gathered.  The per-rank GPU
fit is replaced by a deterministic host stub, so what runs here is everything around it:
the shard assignment, the tables each rank builds, the gather and the reassembly."""
import copy
import os
import socket
import sys

import numpy as np
import pytest

from golden_util import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


# ---- grid_chisq -------------------------------------------------------------------------
def _stub_grid(gu):
    """Replace the device parts of grid_chisq: the upload (host layout only) and the batch
    fit (chi2 a fixed function of each point's table; the 'fitted' table shifts DM)."""
    from pint_amd.engine import build_layout

    def session(model, parnames, toas, gls, npipe=1):
        base = copy.deepcopy(model)
        for p in parnames:
            base[p].frozen = True
        return [(None, build_layout(base, toas, use_gls_basis=gls))] * npipe

    def fit_block(s, lay, grid, mode, down, fitargs, want):
        from golden_util import grid_tables
        tabs = grid_tables(lay, grid)  # (what pint_set_grid forms on the device)
        f0 = tabs[:, lay.offsets["F0"]] + tabs[:, lay.offsets["F0"] + 1]
        f1 = tabs[:, lay.offsets["F1"]] + tabs[:, lay.offsets["F1"] + 1]
        chi2 = (f0 - 61.4854765543) ** 2 * 1e18 + (f1 + 1.18e-15) ** 2 * 1e30 + 60.0
        chi2[f1 < -1.1855e-15] = np.nan  # failed points: a fixed F1 cut
        ft = tabs.copy()
        ft[:, lay.offsets["DM"]] += np.arange(len(tabs)) * 0.0  # unchanged DM
        return chi2, ft

    gu._grid_session = session
    gu._fit_block = fit_block


def _grid_args():
    model, toas, z, meta = load("ngc6440e")
    from pint_amd import WLSFitter
    f = WLSFitter(toas, model)
    g0 = z["grid_F0_hi"].astype(np.longdouble) + z["grid_F0_lo"]
    g1 = z["grid_F1_hi"].astype(np.longdouble) + np.linspace(-1e-17, 1e-17, 5)
    return f, (g0, g1)


def _grid_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import pint_amd.gridutils as gu
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _stub_grid(gu)
        f, vals = _grid_args()
        c2, ex = gu.grid_chisq(f, ("F0", "F1"), vals, extraparnames=["DM"])
        best = gu.best_point(c2, ("F0", "F1"), vals)
        q.put((rank, (c2, ex["DM"], best[0], best[2])))
    finally:
        dist.destroy_process_group()


def test_grid_chisq_two_ranks_gloo():
    out = _spawn(_grid_worker)
    import pint_amd.gridutils as gu
    _stub_grid(gu)
    f, vals = _grid_args()
    want, wex = gu.grid_chisq(f, ("F0", "F1"), vals, extraparnames=["DM"])  # one process
    wbest = gu.best_point(want, ("F0", "F1"), vals)
    assert want.shape == (5, 5) and wex["DM"].shape == (5, 5)
    for rank, (c2, dm, bk, bc) in out.items():
        np.testing.assert_array_equal(c2, want)
        np.testing.assert_array_equal(dm, wex["DM"])
        assert bk == wbest[0] and bc == wbest[2]
    assert np.isnan(want).any() and not np.isnan(want).all()


_FUNCS = (lambda x, y: x, lambda x, y: -x / 2 / y)


def _tuple_args():
    f, (g0, g1) = _grid_args()
    pts = list(zip(g0[[0, 3, 1, 4, 2, 2, 0]], g1[[4, 0, 3, 1, 2, 0, 1]]))   # 7 points: blocks 4 + 3
    tau = -g0[2] / (2 * g1[[0, 1, 2, 3, 4, 2, 1]])
    dpts = list(zip(g0[[0, 1, 2, 3, 4, 0, 1]], tau))
    return f, pts, dpts


def _tuple_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import pint_amd.gridutils as gu
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _stub_grid(gu)
        f, pts, dpts = _tuple_args()
        c2, ex = gu.tuple_chisq(f, ("F0", "F1"), pts, extraparnames=["DM"])
        d2, out, dex = gu.tuple_chisq_derived(f, ("F0", "F1"), _FUNCS, dpts, extraparnames=["DM"])
        g0 = np.unique([p[0] for p in dpts])
        gd, gout, gex = gu.grid_chisq_derived(f, ("F0", "F1"), _FUNCS, (g0, np.unique([p[1] for p in dpts])))
        q.put((rank, (c2, ex["DM"], d2, dex["DM"], gd)))
    finally:
        dist.destroy_process_group()


def test_tuple_chisq_two_ranks_gloo():
    """tuple_chisq / tuple_chisq_derived / grid_chisq_derived (gridutils.py:588/:773/:392)
    split into contiguous per-rank blocks and all-gathered: every rank returns exactly the
    one-process result, in list order."""
    out = _spawn(_tuple_worker)
    import pint_amd.gridutils as gu
    _stub_grid(gu)
    f, pts, dpts = _tuple_args()
    want, wex = gu.tuple_chisq(f, ("F0", "F1"), pts, extraparnames=["DM"])
    assert want.shape == (7,) and wex["DM"].shape == (7,)
    # a tuple list is the same fit as the grid points it names
    for k, (x, y) in enumerate(pts):
        one, _ = gu.grid_chisq(f, ("F0", "F1"), (np.array([x]), np.array([y])))
        np.testing.assert_array_equal(one.reshape(-1), want[k:k + 1])
    dwant, dout, dwex = gu.tuple_chisq_derived(f, ("F0", "F1"), _FUNCS, dpts, extraparnames=["DM"])
    assert len(dout) == 7 and all(len(o) == 2 for o in dout)
    for (x, y), o in zip(dpts, dout):
        assert o[0] == x and o[1] == -x / 2 / y
    g0 = np.unique([p[0] for p in dpts])
    gt = np.unique([p[1] for p in dpts])
    gwant, gout, _ = gu.grid_chisq_derived(f, ("F0", "F1"), _FUNCS, (g0, gt))
    assert gwant.shape == (len(gt), len(g0)) and gout[1].shape == gwant.shape
    G0, GT = np.meshgrid(g0, gt)
    np.testing.assert_array_equal(gout[1], -G0 / 2 / GT)
    for rank, (c2, dm, d2, ddm, gd) in out.items():
        np.testing.assert_array_equal(c2, want)
        np.testing.assert_array_equal(dm, wex["DM"])
        np.testing.assert_array_equal(d2, dwant)
        np.testing.assert_array_equal(ddm, dwex["DM"])
        np.testing.assert_array_equal(gd, gwant)
    assert np.isnan(want).any() and not np.isnan(want).all()


# ---- PTA sharding -------------------------------------------------------------------------
def test_lpt_shard_properties():
    from pint_amd.pta import lpt_shard
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        costs = list(rng.uniform(1, 10, 68))
        sh = lpt_shard(costs, world)
        flat = sorted(i for s in sh for i in s)
        assert flat == list(range(68))
        loads = [sum(costs[i] for i in s) for s in sh]
        # LPT bound: makespan <= 4/3 of optimal, and optimal >= mean load
        assert max(loads) <= 4 / 3 * max(np.mean(loads), max(costs)) + 1e-9
        assert sh == lpt_shard(costs, world)  # deterministic


def _pta_items():
    items = []
    for k, name in enumerate(["pta_iso", "pta_ell1", "pta_dd", "ngc6440e", "j0740"]):
        model, toas, z, meta = load(name)
        items.append((model, toas))
    return items


def _stub_fit(items, mode, downhill, maxiter, **kw):
    """Host stand-in for the per-rank batched fit: moves every free parameter by a fixed
    fraction of its uncertainty and reports a chi2 that identifies the pulsar."""
    from pint_amd.fitter import FitResult
    out = []
    for model, toas in items:
        r = FitResult()
        for p in model.free_params:
            par = model[p]
            e = par.uncertainty or 1e-9
            v = np.longdouble(par.value) + np.longdouble(0.25 * e)
            par.value = v if (par.long_double or par.kind == "mjd") else float(v)  # as unpack_table
            par.uncertainty = 0.5 * e
        r.chi2 = float(toas.ntoas) + 0.5
        r.status = "converged"
        r.converged = True
        out.append(r)
    return out


def _pta_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from pint_amd.pta import fit_pta
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        items = _pta_items()
        res, shards = fit_pta(items, mode="gls", fit_fn=_stub_fit)
        vals = [[(float(m[p].value), float(np.longdouble(m[p].value) - np.longdouble(float(m[p].value))),
                  m[p].uncertainty) for p in m.free_params] for m, _ in items]
        q.put((rank, ([r.chi2 for r in res], [r.status for r in res], vals, shards)))
    finally:
        dist.destroy_process_group()


def test_fit_pta_two_ranks_gloo():
    from pint_amd.pta import fit_pta
    out = _spawn(_pta_worker)
    items = _pta_items()
    res, shards1 = fit_pta(items, mode="gls", fit_fn=_stub_fit)  # one process
    want_vals = [[(float(m[p].value), float(np.longdouble(m[p].value) - np.longdouble(float(m[p].value))),
                   m[p].uncertainty) for p in m.free_params] for m, _ in items]
    assert shards1 == [list(range(len(items)))]
    sh = out[0][3]
    assert sh == out[1][3] and sorted(sh[0] + sh[1]) == list(range(len(items))) and sh[0] and sh[1]
    for rank, (chi2, status, vals, _) in out.items():
        assert chi2 == [r.chi2 for r in res]
        assert status == ["converged"] * len(items)
        assert vals == want_vals  # every rank holds every fitted model, to the dd pair
