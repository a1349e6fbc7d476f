"""Benchmark: GLS fits/s on the synthetic 68-pulsar x 10k-TOA PTA (BASELINE.json metric),
plus chi2-grid points/s, on N MI355X GPUs of one node.

One *step* = one GLSFitter.fit_toas(maxiter=1) (fitter.py:2104) of every pulsar of a
68-pulsar PTA, batched in one launch sequence per GPU: design matrix + residuals
(k_eval/k_resid), Gram on FP64 MFMA (k_gram_v, + trig sums k_trig), Cholesky/solve/
covariance (k_solve_dmx), double-double parameter update (k_apply), post-fit residuals and
Woodbury chi2 (k_wdot/k_wsolve), with the fit outputs (steps, errors, covariances, chi2)
copied back to the host (on a copy stream, overlapped with the kernels).  Weak scaling: rank r fits its own 68-pulsar PTA (pulsar seeds 68r .. 68r+67),
no data-path collective; the max over ranks is the step time and value = 68 x N / step.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)
MI355X_FP64_MFMA_PEAK_TFLOPS = 78.6  # vendor FP64 matrix peak


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--npsr", type=int, default=68)
    ap.add_argument("--ntoas", type=int, default=10000)
    ap.add_argument("--grid", type=int, default=256, help="grid side for the chi2-grid leg (0 = skip)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--j0740", type=int, default=256,
                    help="(M2, SINI) grid side of the C3/C4 J0740 legs (0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    from pint_amd.engine import Session, build_layout, pack_table
    from pint_amd.simulation import make_pta

    # ---- workload: this rank's own PTA (weak scaling; pulsar i uses seed i) ----
    mine = list(range(rank * args.npsr, (rank + 1) * args.npsr))
    t0 = time.time()
    from pint_amd import simulation as sim
    from pint_amd.timing_model import get_model
    specs = []
    for i in mine:
        kind = "ELL1" if i % 6 in (1, 4) else ("DD" if i % 6 == 2 else "")
        m = get_model(sim.pta_par(i, kind))
        specs.append(dict(model=m, start=53000, end=56652, ntoas=args.ntoas, freq=[800, 1200, 1600, 2000],
                          obs="geocenter", error_us=0.5, add_noise=True, add_correlated_noise=True, seed=i))
    toas = sim.make_fake_toas_batch(specs)
    items = [(sp["model"], t) for sp, t in zip(specs, toas)]
    log(f"[rank {rank}] generated {len(items)} pulsars x {args.ntoas} TOAs in {time.time()-t0:.1f}s")

    s = Session(device=local)
    lays = [s.add(build_layout(m, t)) for m, t in items]
    tabs0 = [pack_table(l, m) for l, (m, _) in zip(lays, items)]
    s.set_instances(list(zip(lays, tabs0)))
    flat0 = np.concatenate(tabs0)
    nin = len(lays)
    ones = np.ones(nin)

    s.set_lazy(True)

    def step():
        s.set_tables(flat0)
        s.eval(want_M=Session.FIT)
        s.fit_step(1)
        out = s.read_step()    # steps, errors, timing covariance -> host (fit outputs)
        s.apply_step(ones)
        s.eval(want_M=False)
        c2 = s.chi2_gls()      # post-fit GLS chi2 (GLSFitter returns calc_chi2())
        return out, c2

    SLOT_GRAM = 6
    s.set_timing_mask(1 << SLOT_GRAM)  # timed region: HIP events around the Gram kernel only

    def run(nsteps):
        """nsteps steps, pipelined two deep: step k+1 is enqueued before the host waits for
        step k (Session.step_end / check_step), so the device does not idle while the host
        checks a step and issues the next.  Returns the summed Gram-kernel event time."""
        kt, prev = 0.0, None
        for _ in range(nsteps):
            step()
            cur = s.step_end()
            if prev is not None:
                s.check_step(prev)  # device status + the Gram kernel's HIP-event time
                kt += s.timing()[SLOT_GRAM]
            prev = cur
        if prev is not None:
            s.check_step(prev)
            kt += s.timing()[SLOT_GRAM]
        return kt

    run(args.warmup)
    barrier()
    t0 = time.perf_counter()
    kt_gram = run(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kt_gram /= args.steps
    ms_step = dt / args.steps * 1e3
    # per-kernel breakdown: a separate instrumented pass (every timing slot's events on; they
    # cost ~5 us each, so this pass is not the timed one)
    s.set_timing_mask(0xFF)
    kt = np.zeros(8)
    nprof = 3
    for _ in range(nprof):
        step()
        s.check()
        kt += s.timing()
    kt /= nprof
    fits_per_s = args.npsr * world / (dt / args.steps)

    # ---- roofline: work per launch / HIP-event time of that kernel ----
    K = np.array([l.K for l in lays])                # timing + red-noise columns
    P = np.array([len(l.columns) for l in lays])     # timing columns
    N = np.array([l.n for l in lays]).astype(float)
    R = K - P
    vl = [s.vgram_layout(l) for l in lays]
    # k_gram_v: MFMA tiles [T|r|DMX slots] x [T|r|slots|F] of 16x16 + the trig tile A^T B,
    # 2048 flops per tile per 4 rows
    tiles = []
    for vg, ns, kpv, r0 in vl:
        ntr, nt = (r0 + 1 + ns) // 16, kpv // 16
        tiles.append(ntr * nt - ntr * (ntr - 1) // 2 + 1 if vg else 0)
    tiles = np.array(tiles, dtype=float)
    flops = {
        "k_gram": float(np.sum(tiles * N * 512.0)),           # FP64 MFMA flops executed
        "k_solve": float(np.sum(K.astype(float) ** 3)),       # chol K^3/3 + inverse/cov 2K^3/3
    }
    # the full GLS Gram the reference forms (2 N K^2, SURVEY.md 8(d) F_gram) for reference
    gram_equiv = float(np.sum(2.0 * N * (K + 1.0) ** 2))
    nbytes = {
        "k_eval_M": float(np.sum(N * (120 + 8 * P))),          # SURVEY.md 8(d) B_dm
        "k_eval": float(np.sum(N * (120 + 8))),                # B_res
        "k_resid": float(np.sum(N * (8 * 4 + 8 * 2))),        # phase hi/lo, ftaylor, sigma in; resid out
        "k_woodbury": float(np.sum(N * (8 * 4))),              # r, sigma, fundamental (cos, sin) in
    }
    names = ["k_eval", "k_resid", "gram_span", "k_solve", "k_eval_M", "k_woodbury", "k_gram", "k_greduce"]
    kms = {n: float(v) for n, v in zip(names, kt)}
    dom = max((n for n in names if n not in ("gram_span", "k_greduce")), key=lambda n: kms[n])
    if dom == "k_gram":
        kms[dom] = kt_gram  # the dominant kernel's time from the timed region itself
    peaks = load_peaks()
    if kms[dom] <= 0:  # no per-kernel events (PINT_NO_EVENTS)
        roof = {"kernel": dom, "bound": None, "achieved": None, "peak": None, "unit": None, "frac": None}
    elif dom in flops:
        ach = flops[dom] / (kms[dom] * 1e-3) / 1e12
        pk = MI355X_FP64_MFMA_PEAK_TFLOPS
        roof = {"kernel": "k_gram_v" if dom == "k_gram" else dom, "bound": "mfma" if dom == "k_gram" else "fp64",
                "achieved": round(ach, 3), "peak": pk, "unit": "TFLOP/s", "frac": round(ach / pk, 4)}
    else:
        ach = nbytes[dom] / (kms[dom] * 1e-3) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": MI355X_HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / MI355X_HBM_PEAK_GBS, 4)}
    roof["traffic"] = pmc_traffic(roof["kernel"], args)
    roof["kernel_ms"] = {n: round(v, 4) for n, v in kms.items()}
    roof["kernel_ms_source"] = ("k_gram: HIP events in the timed region; others: a separate instrumented pass "
                                f"of {nprof} steps (gram_span = ecorr + Gram + reduction)")
    roof["per_kernel"] = {}
    for n in names:
        if kms[n] <= 0:
            continue
        if n in flops:
            roof["per_kernel"][n] = {"TFLOP/s": round(flops[n] / (kms[n] * 1e-3) / 1e12, 3)}
        if n in nbytes:
            roof["per_kernel"][n] = {"GB/s": round(nbytes[n] / (kms[n] * 1e-3) / 1e9, 1)}
    if kms["k_gram"] > 0:
        roof["gram_full_equiv_tflops"] = round(gram_equiv / (kms["k_gram"] * 1e-3) / 1e12, 2)
    if peaks:
        roof["measured_peaks"] = peaks

    # ---- chi2-grid leg (C4 shape: 256x256 (F0,F1) WLS grid of the NGC6440E fixture) ----
    grid = None
    if args.grid > 0:
        grid = grid_leg(args.grid, rank, world, dist, barrier)

    j0740 = None
    if args.j0740 > 0:
        j0740 = j0740_legs(args.j0740, rank, world, dist, barrier)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu = cpu_baseline(items[:1])

    if rank == 0:
        out = {"metric": "GLS fits/sec, 68-PSR x 10k-TOA synthetic PTA (whole node)", "value": round(fits_per_s, 3),
               "unit": "fits/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f64+dd", "data": "synthetic (make_fake_toas-style, GPU-zeroed)",
               "config": {"workload": f"pta{args.npsr}x{args.ntoas // 1000}k GLSFitter maxiter=1 per GPU",
                          "npsr": args.npsr, "npsr_total": args.npsr * world, "ntoas": args.ntoas,
                          "K_cols_max": int(K.max() - 1),
                          "parallelism": f"one PTA per GPU x{world} (weak)"},
               "roofline": roof, "grid": grid, "j0740": j0740, "cpu_baseline": cpu}
        print(json.dumps(out))
    s.close()
    if dist is not None:
        dist.destroy_process_group()


def load_peaks():
    """Peaks measured on an MI355X by bench/peaks.hip (committed under profiles/)."""
    f = os.path.join(ROOT, "profiles", "peaks_r01.json")
    if os.path.exists(f):
        with open(f) as fh:
            return json.load(fh)
    return None


def pmc_traffic(kernel, args):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this
    same bench command (FETCH_SIZE x2 on gfx950 per MI355X_MICROARCH.md, + WRITE_SIZE)."""
    f = os.path.join(ROOT, "profiles", "pmc_r01.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        d = json.load(fh)
    if d.get("workload") != f"pta{args.npsr}x{args.ntoas}":
        return None
    k = d.get("kernels", {}).get(kernel)
    return None if k is None else k.get("hbm_bytes")


def grid_leg(side, rank, world, dist, barrier):
    """chi2 over a side x side (F0, F1) grid, WLSFitter per point (gridutils.py:166 parallel
    semantics), points sharded over ranks; timed over one full grid."""
    import copy
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import load
    from pint_amd import WLSFitter
    from pint_amd.gridutils import grid_chisq
    model, toas, _, _ = load("ngc6440e")
    f = WLSFitter(toas, model)
    f.fit_toas(maxiter=1)
    F0, F1 = np.longdouble(f.model.F0.value), np.longdouble(f.model.F1.value)
    s0, s1 = f.model.F0.uncertainty, f.model.F1.uncertainty
    g0 = F0 + np.linspace(-3, 3, side) * np.longdouble(s0)
    g1 = F1 + np.linspace(-3, 3, side) * np.longdouble(s1)
    grid_chisq(f, ("F0", "F1"), (g0, g1))  # warm-up: the TOAs uploaded, batch buffers allocated
    barrier()
    t0 = time.perf_counter()
    chi2, _ = grid_chisq(f, ("F0", "F1"), (g0, g1))
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return {"metric": "chi2-grid points/sec", "value": round(side * side / dt, 1), "unit": "points/s",
            "workload": f"NGC6440E (62 TOAs) {side}x{side} (F0,F1) WLSFitter", "seconds": round(dt, 3),
            "chi2_min": float(np.nanmin(chi2))}


def j0740_data():
    """C3 data: J0740+6620 (ELL1 + Shapiro, 68 DMX, ECORR) on 50k synthetic TOAs
    (make_fake_toas_uniform 56640-58461, 820/1400 MHz alternating, 1 us, noise, flags
    -f Rcvr1_2_GUPPI -fe Rcvr1_2, seed 0), empty DMX/JUMP masks frozen (the reference's
    find_empty_masks(freeze=True) step of the C3 setup)."""
    from pint_amd import simulation as sim
    from pint_amd.timing_model import get_model
    model = get_model(os.path.join(ROOT, "tests", "golden", "J0740+6620.par"))
    toas = sim.make_fake_toas_uniform(56640, 58461, 50000, model, freq=[820.0, 1400.0], obs="geocenter",
                                      error=1.0, add_noise=True, flags={"f": "Rcvr1_2_GUPPI", "fe": "Rcvr1_2"},
                                      seed=0)
    mjd = toas.get_mjds()
    frozen = []
    for n in model.dmx_params():
        tag = n.split("_")[1]
        r1, r2 = float(model["DMXR1_" + tag].value), float(model["DMXR2_" + tag].value)
        if not np.any((mjd >= r1) & (mjd <= r2)):
            model[n].frozen = True
            frozen.append(n)
    for n in model.mask_params("JUMP"):
        p = model[n]
        if len(toas.select_mask(p.key, p.key_value)) == 0:
            p.frozen = True
            frozen.append(n)
    return model, toas, frozen


def j0740_legs(side, rank, world, dist, barrier):
    """C3 and the second C4 shape on j0740_data().  C3: one
    DownhillGLSFitter(maxiter=10) fit, timed.  C4: grid_chisq over (M2, SINI) side x side,
    M2 in [0.2, 0.3] Msun, SINI = sin(86.25..88.5 deg) (profiling/bench_chisq_grid.py:33-35),
    GLSFitter per point, sharded over ranks."""
    import copy
    from pint_amd import DownhillGLSFitter, GLSFitter
    from pint_amd.fitter import MaxiterReached
    from pint_amd.gridutils import grid_chisq
    model, toas, frozen = j0740_data()
    out = {"workload": "J0740+6620 synthetic 50k TOAs (C3)", "free_params": len(model.free_params),
           "frozen_empty": len(frozen)}
    f = DownhillGLSFitter(toas, copy.deepcopy(model))
    try:
        f.fit_toas(maxiter=10)  # warm-up (library load, first-call allocations)
    except MaxiterReached:
        pass
    barrier()
    f = DownhillGLSFitter(toas, copy.deepcopy(model))
    t0 = time.perf_counter()
    try:
        f.fit_toas(maxiter=10)
        conv = True
    except MaxiterReached:
        conv = False
    dt = time.perf_counter() - t0
    out["downhill_gls"] = {"metric": "DownhillGLSFitter fits/sec (maxiter=10)", "value": round(1.0 / dt, 3),
                           "seconds": round(dt, 4), "converged": conv, "chi2": float(f.resids.chi2)}
    g = GLSFitter(toas, copy.deepcopy(model))
    g.fit_toas(maxiter=1)
    m2 = np.linspace(0.2, 0.3, side)
    sini = np.sin(np.deg2rad(np.linspace(86.25, 88.5, side)))
    grid_chisq(g, ("M2", "SINI"), (m2, sini))  # warm-up (first-touch of the batch buffers)
    barrier()
    t0 = time.perf_counter()
    chi2, _ = grid_chisq(g, ("M2", "SINI"), (m2, sini))
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    out["grid_m2_sini"] = {"metric": "chi2-grid points/sec", "value": round(side * side / dt, 1),
                           "unit": "points/s", "workload": f"J0740 50k TOAs {side}x{side} (M2,SINI) GLSFitter",
                           "seconds": round(dt, 3), "chi2_min": float(np.nanmin(chi2))}
    return out


def cpu_baseline(items):
    """The oracle (numpy longdouble restatement, oracle/pint_oracle.py) timed on this host
    on a bounded sample: GLS fits of one 10k-TOA PTA pulsar, scaled to fits/s."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pint_oracle as O
    except Exception as e:  # oracle missing: report, never fall back
        return {"value": None, "error": repr(e)}
    model, toas = items[0]
    try:
        from threadpoolctl import threadpool_limits
        lim = threadpool_limits(1)
    except Exception:
        lim = None
    t0 = time.perf_counter()
    nfit = 0
    while True:
        O.gls_fit_from_product_inputs(model, toas)
        nfit += 1
        if time.perf_counter() - t0 > 12.0 or nfit >= 200:
            break
    dt = time.perf_counter() - t0
    if lim is not None:
        lim.unregister() if hasattr(lim, "unregister") else None
    return {"value": round(nfit / dt, 4), "unit": "fits/s", "cores": 1, "kind": "port",
            "sample": f"{nfit} GLS fit(s) (maxiter=1 + post-fit GLS chi2) of one {toas.ntoas}-TOA PTA pulsar "
                      f"(K={len(model.free_params)+1} + {2 * (model.red_noise_params()[2])} red-noise columns), "
                      f"numpy longdouble oracle, BLAS limited to 1 thread, {dt:.1f} s"}


if __name__ == "__main__":
    main()
