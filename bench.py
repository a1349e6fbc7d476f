"""Benchmark: GLS fits/s on the synthetic 68-pulsar x 10k-TOA PTA (BASELINE.json metric),
plus chi2-grid points/s, on N MI355X GPUs of one node.

One *step* = one GLSFitter.fit_toas(maxiter=1) (fitter.py:2104) of every pulsar of a rank's
shard, batched in one launch sequence per GPU: design matrix + residuals (k_eval/k_resid),
Gram on FP64 MFMA (k_gram_v), Cholesky/solve/covariance (k_solve_dmx; iterative refinement
where the condition estimate asks for it), double-double parameter update (k_apply), post-fit residuals and Woodbury
chi2 (k_resid2's trig tiles + k_wsolve), with the fit outputs (steps, errors, covariances, chi2) copied back
to the host on a copy stream, overlapped with the kernels.

Sharding (pint_amd.pta): the pulsars are assigned to ranks by
longest-processing-time on the fit cost N K^2 + 8 N P; there is no data-path collective.
* value ("scaling": "strong"): the configured 68-pulsar PTA split over the N ranks
  (north_star's target); value = 68 / max-over-ranks step time.
* pta_weak (N > 1): a PTA of 68 x N pulsars (pulsar i uses seed i) over N ranks, ~68 per GPU.

The step includes the noise realisations GLSFitter.fit_toas computes when full_cov=False
(fitter.py:2269-2282): k_noise_red after the solve, the per-pulsar arrays copied to the host.

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
SLOT_GRAM = 6                      # pint_last_timing slot of the Gram kernels
GRAM_EVERY = 8                     # Gram timing events on every 8th timed step


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # 0.5 ms each: steady state, not the first steps
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--npsr", type=int, default=68)
    ap.add_argument("--ntoas", type=int, default=10000)
    ap.add_argument("--grid", type=int, default=256, help="grid side for the chi2-grid leg (0 = skip)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--weak", type=int, default=1, help="also time a 68 x N pulsar PTA over the N ranks (N > 1)")
    ap.add_argument("--c2", type=int, default=256, help="B1855 (C2) fits per batched step (0 = skip the C2 leg)")
    ap.add_argument("--j0740", type=int, default=256,
                    help="(M2, SINI) grid side of the C3/C4 J0740 legs (0 = skip)")
    ap.add_argument("--emulate-world", default="2,4,8",
                    help="N=1 only: time every rank's LPT shard of the PTA for these world sizes on this "
                         "GPU, one after the other (predicted_strong; '' = skip)")
    ap.add_argument("--graph", default="0", choices=["0", "1", "auto"],
                    help="step launches: 0 enqueued from the host, 1 one HIP-graph replay per step, auto the "
                         "faster of the two on a short trial (every rank makes the same choice)")
    ap.add_argument("--pipes", default="auto",
                    help="independent step pipelines per GPU (sessions with their own streams and buffers, fed "
                         "round-robin): a count, or auto = the fastest of 1..--max-pipes on a short trial")
    ap.add_argument("--max-pipes", type=int, default=2)
    ap.add_argument("--cold-start", type=int, default=1,
                    help="N=1 only: upload + first fit of the PTA in a fresh session (cold_start)")
    args = ap.parse_args()

    # (several pipelines share the process's GPU_MAX_HW_QUEUES hardware queues, default 4:
    # measured, 2 x 9-pulsar pipelines 0.105 ms per step with 4 queues, 0.237 with 12, where
    # the hardware scheduler time-slices the queues; the variable is left as it is)
    from pint_amd import _lib
    _lib.lib()  # the process's HIP runtime (the system ROCm's), before torch is imported
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a box with fewer GPUs than ranks (not the measured
    # configuration): PINT_BENCH_SHARE_GPU=1 maps rank r to GPU r mod (GPUs), and
    # PINT_BENCH_BACKEND=gloo carries the collectives on the host (RCCL refuses two ranks on
    # one GPU).  The driver's N-GPU runs use neither.
    backend = os.environ.get("PINT_BENCH_BACKEND", "nccl")
    if world > 1 and os.environ.get("PINT_BENCH_SHARE_GPU") == "1":
        import torch
        local = local % max(1, torch.cuda.device_count())
        os.environ["LOCAL_RANK"] = str(local)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method="env://")

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(v):
        if dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    from pint_amd import simulation as sim
    from pint_amd.pta import fit_cost, lpt_shard

    # ---- value ("scaling": "strong"): the configured 68-pulsar PTA, LPT-sharded over the N
    # ranks (north_star: the 68-pulsar x 10k-TOA PTA at 1/2/4/8 GPUs) ----
    models = [sim.pta_model(i) for i in range(args.npsr)]
    costs = [fit_cost(m, n=args.ntoas) for m in models]
    shards = lpt_shard(costs, world)
    leg = pta_leg(shards[rank], models, args, rank, barrier, max_over_ranks, profile=True)
    fits_per_s = args.npsr / (leg["dt"] / args.steps)
    weak = None
    if world > 1 and args.weak:
        # extra: weak scaling, a 68 x N pulsar PTA (pulsar i uses seed i), ~68 per rank
        ntot = args.npsr * world
        models_w = models + [sim.pta_model(i) for i in range(args.npsr, ntot)]
        costs_w = costs + [fit_cost(m, n=args.ntoas) for m in models_w[args.npsr:]]
        sh2 = lpt_shard(costs_w, world)
        leg2 = pta_leg(sh2[rank], models_w, args, rank, barrier, max_over_ranks, profile=False)
        weak = {"metric": f"GLS fits/sec, a {ntot}-pulsar PTA over {world} ranks (~{args.npsr} per GPU, weak scaling)",
                "value": round(ntot / (leg2["dt"] / args.steps), 3), "unit": "fits/s",
                "ms_per_step": round(leg2["dt"] / args.steps * 1e3, 4),
                "pulsars_per_rank": [len(s) for s in sh2]}

    roof = leg["roofline"]
    cold = cold_start(leg["items"], rank) if (world == 1 and args.cold_start) else None
    emu = None
    if world == 1 and args.emulate_world:
        emu = emulate_world(leg["items"], costs, [int(x) for x in args.emulate_world.split(",") if x],
                            args, fits_per_s, leg["dt"] / args.steps)
    grid = grid_leg(args.grid, dist, barrier, max_over_ranks) if args.grid > 0 else None
    j0740 = j0740_legs(args.j0740, dist, barrier, max_over_ranks) if args.j0740 > 0 else None
    c2 = c2_leg(args.c2, 20, 3, world, barrier, max_over_ranks, npipes(args)) if args.c2 > 0 else None
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu = cpu_baseline(leg["items"])

    if rank == 0:
        out = {"metric": "GLS fits/sec, 68-PSR x 10k-TOA synthetic PTA (whole node)", "value": round(fits_per_s, 3),
               "unit": "fits/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(leg["dt"] / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
               "vs_baseline": None, "dtype": "f64+dd",
               "data": "synthetic (make_fake_toas-style PTA, TOAs generated and zeroed on the GPU)",
               "config": {"workload": f"pta{args.npsr}x{args.ntoas // 1000}k GLSFitter.fit_toas(maxiter=1) incl. noise "
                                      f"realisations (the {args.npsr}-pulsar PTA, LPT-sharded over {world} rank(s))",
                          "npsr": args.npsr, "ntoas": args.ntoas,
                          "pulsars_per_rank": [len(s) for s in shards], "K_cols_max": leg["kmax"],
                          "launch": leg["launch"], "pipelines": leg["pipes"],
                          "parallelism": f"pulsar shards x{world} (LPT, no data-path collective)"},
               "roofline": roof, "pta_weak": weak, "predicted_strong": emu, "cold_start": cold,
               "grid": grid, "j0740": j0740, "c2": c2,
               "cpu_baseline": cpu}
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def pta_leg(mine, models, args, rank, barrier, max_over_ranks, profile):
    """Time K steps (GLSFitter maxiter=1 of every pulsar in `mine`) on this rank's GPU;
    returns the max-over-ranks wall time and, with profile, the roofline record."""
    from pint_amd import simulation as sim
    from pint_amd.engine import Session, build_layout, pack_table
    t0 = time.time()
    items = sim.make_pta(ntoas=args.ntoas, indices=mine, models=[models[i] for i in mine])
    log(f"[rank {rank}] generated {len(items)} pulsars x {args.ntoas} TOAs in {time.time() - t0:.1f}s")
    ss, lays = pipelines(items, npipes(args))
    dt, kt_gram, n_gram, step, launch, p = timed_steps(ss, args.steps, args.warmup, barrier, max_over_ranks,
                                                       graph=args.graph, pipes=args.pipes)
    out = {"dt": dt, "items": items, "kmax": int(max(l.K for l in lays)), "launch": launch, "pipes": p}
    if profile:
        out["roofline"] = roofline(ss[0], lays, kt_gram / max(1, n_gram), step, args)
        out["roofline"]["gram_event_launches"] = int(n_gram)
    for s in ss:
        s.close()
    return out


def npipes(args):
    return args.max_pipes if args.pipes == "auto" else max(1, int(args.pipes))


def pipelines(items, n):
    """n sessions (independent pipelines: streams, device buffers) holding the same batch;
    returns them and the first one's layouts."""
    from pint_amd.engine import Session, pack_table
    ss, lays0 = [], None
    for _ in range(n):
        s = Session(device=int(os.environ.get("LOCAL_RANK", "0")))
        lays = s.add_all(items)
        s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
        ss.append(s)
        lays0 = lays0 or lays
    return ss, lays0


def emulate_world(items, costs, worlds, args, value1, step1):
    """Predicted strong scaling of the headline metric on this one GPU: for each world size N,
    every rank's LPT shard (pint_amd.pta.lpt_shard, the assignment bench.py uses at N ranks)
    is uploaded into its own session and timed for the same K steps, one shard after the
    other; the predicted N-GPU step is the slowest shard's (the max-over-ranks the N-rank run
    takes).  Host-side enqueue runs on this one process as it would on each rank."""
    from pint_amd.engine import Session, build_layout, pack_table
    from pint_amd.pta import lpt_shard

    def nobarrier():
        pass

    steps, warm = max(20, args.steps // 2), max(3, args.warmup // 2)
    out = {"method": ("each rank's LPT shard timed alone on this GPU (same step as the headline), "
                      f"median of 3 runs of {steps} steps after {warm} warm-up; predicted value = npsr / "
                      "max over shards"),
           "n1": {"value": round(value1, 3), "ms_per_step": round(step1 * 1e3, 4)}}
    for nw in worlds:
        if nw <= 1:
            continue
        per, modes = [], []
        for sh in lpt_shard(costs, nw):
            if not sh:
                per.append(0.0)
                modes.append(None)
                continue
            ss, _ = pipelines([items[i] for i in sh], npipes(args))
            # the median of three timed runs: one host hiccup in a short run would otherwise
            # stand for the shard (a 4x outlier seen once in ~20 runs)
            reps = []
            for _ in range(3):
                dt, _, _, _, launch, p = timed_steps(ss, steps, warm, nobarrier, lambda v: v, graph=args.graph,
                                                     gram_pass=False, pipes=args.pipes)
                reps.append(dt / steps)
            for s in ss:
                s.close()
            per.append(float(np.median(reps)))
            modes.append(f"{launch} x{p}")
        mx = max(per)
        out[f"n{nw}"] = {"value": round(len(items) / mx, 3), "ms_per_step": round(mx * 1e3, 4),
                         "ms_per_shard": [round(p * 1e3, 4) for p in per],
                         "pulsars_per_rank": [len(sh) for sh in lpt_shard(costs, nw)], "launch": modes,
                         "speedup_vs_n1": round(step1 / mx, 3)}
        log(f"[emulate {nw}] shards {[round(p * 1e3, 3) for p in per]} ms -> {len(items) / mx:.0f} fits/s")
    return out


def cold_start(items, rank):
    """Cold start of the PTA (the library already loaded): a fresh session, every pulsar's
    host layout and TOA columns with the library's packing and upload beside them
    (Session.add_all), the instances (incl. the per-pulsar set-up kernels), then the first
    GLSFitter.fit_toas(maxiter=1) step of all pulsars, synchronously.  Wall times."""
    from pint_amd.engine import Session, pack_table
    t0 = time.perf_counter()
    s = Session(device=int(os.environ.get("LOCAL_RANK", "0")))
    ts = time.perf_counter()
    lays = s.add_all(items)  # host layouts + TOA columns here, the library's packing/staging beside them
    ta = time.perf_counter()
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
    s.check()
    t2 = time.perf_counter()
    s.eval(want_M=Session.FIT)
    s.fit_step_apply(1, 1.0)
    s.read_step()
    s.noise_resids()
    s.eval(want_M=False)
    s.chi2_gls()
    s.check()
    t3 = time.perf_counter()
    s.close()
    out = {"pulsars": len(items), "session_ms": round((ts - t0) * 1e3, 2),
           "add_all_ms": round((ta - ts) * 1e3, 2),
           "add_all_parts_ms": {"layouts_and_columns": round(s.add_timing["host_ms"], 2),
                                "upload_wait": round(s.add_timing["upload_wait_ms"], 2)},
           "set_instances_ms": round((t2 - ta) * 1e3, 2),
           "first_fit_ms": round((t3 - t2) * 1e3, 3), "cold_start_ms": round((t3 - t0) * 1e3, 2),
           "note": "wall, host included: host layouts and TOA columns overlapped with the library's packing and "
                   "upload (Session.add_all), the instances and per-pulsar set-up kernels, the first synchronous "
                   "fit step"}
    log(f"[rank {rank}] cold start {out}")
    return out


def timed_steps(sessions, steps, warmup, barrier, max_over_ranks, graph="auto", gram_pass=True, pipes=1):
    """Time `steps` fit steps of the batch (warm-up first); one step is
    GLSFitter.fit_toas(maxiter=1) of every instance from its initial model.

    sessions: one Session, or several holding the same batch -- independent pipelines
    (each its own streams and device buffers) fed round-robin, step i on pipeline i mod P,
    each pipelined L.NSLOT deep: a small batch's step is a chain of latency-bound kernels
    that leaves most of the chip idle, and a second or third pipeline's kernels run in those
    gaps.  pipes: how many of the sessions to use, or "auto": the fastest P on a short trial
    after the warm-up (every rank makes the same choice).
    graph: 0 enqueue every launch of every step from the host; 1 capture the step once per
    pipeline slot into a HIP graph and replay it (the same kernels, copies and outputs, one
    host launch per step); "auto" the faster of the two on the trial.
    Returns (max-over-ranks seconds, summed Gram event time of the sampled steps, their
    count, step, launch mode, pipelines)."""
    from collections import deque
    from pint_amd import _lib as L
    from pint_amd.engine import Session
    if isinstance(sessions, Session):
        sessions = [sessions]
    for s in sessions:
        s.save_tables()        # the initial models, resident in HBM like the TOAs
        s.set_lazy(True)
        # Gram timing: HIP events on the Gram dispatches only (hipExtLaunchKernel start/stop
        # on its first/last dispatch packet, or marker packets on the other Gram paths), on
        # every GRAM_EVERY-th step of a pass of enqueued steps run after the timed region (the
        # first pipeline alone): an event pair still idles the stream ~5-10 us (a 9-pulsar
        # step's trace shows it), so the timed steps carry none.
        s.set_timing_mask(0)
        s.set_timing_every(GRAM_EVERY)

    def step_calls(s):
        """The step as separate library calls (the graph capture records these)."""
        s.restore_tables()     # every step fits from the initial models (device->device copy)
        s.eval(want_M=Session.FIT)
        s.fit_step_apply(1, 1.0)  # the GLS step and the full-step update (fused into the solve)
        out = s.read_step()    # steps, errors, timing covariance -> host (fit outputs)
        nz = s.noise_resids()  # noise realisations -> host (fitter.py:2269-2282, full_cov=False)
        s.eval(want_M=False)
        c2 = s.chi2_gls()      # post-fit GLS chi2 (GLSFitter returns calc_chi2())
        return out, nz, c2

    def step(s):
        """The same step enqueued by one call (pint_fit_step_enqueue, closes the step);
        returns its slot."""
        return s.fit_step_enqueue(restore=True, lam=1.0)[0]

    def replay(s):
        s.replay()
        return s.step_end()

    def run(nsteps, launch, sess):
        """nsteps steps over the pipelines `sess`, round-robin, each pipelined L.NSLOT deep:
        before a step is enqueued on a pipeline, the step that last used that pipeline's
        slot is checked (Session.check_step), so every device queue holds up to NSLOT - 1
        steps while the host enqueues the next; launch(s) enqueues and closes one step on s
        and returns its slot.  Returns the summed Gram-kernel event time of the sampled
        steps and their count."""
        kt, nk = 0.0, 0
        pend = [deque() for _ in sess]
        # PINT_BENCH_TRACE=1: the host clock after every launch and every check (2 floats per
        # step into a preallocated array), reported on stderr
        tr = np.zeros(2 * nsteps + 2) if os.environ.get("PINT_BENCH_TRACE") else None
        clk = time.perf_counter

        def check_one(k):
            nonlocal kt, nk
            sess[k].check_step(pend[k].popleft())
            t = sess[k].timing()[SLOT_GRAM]
            kt, nk = kt + t, nk + (t > 0)

        for i in range(nsteps):
            k = i % len(sess)
            if len(pend[k]) >= L.NSLOT:
                check_one(k)
            if tr is not None:
                tr[2 * i] = clk()
            pend[k].append(launch(sess[k]))
            if tr is not None:
                tr[2 * i + 1] = clk()
        for k in range(len(sess)):
            while pend[k]:
                check_one(k)
        if tr is not None:
            tr[-1] = clk()
            st = np.diff(tr[0:2 * nsteps:2]) * 1e3                   # launch to launch
            ln = (tr[1:2 * nsteps:2] - tr[0:2 * nsteps:2]) * 1e3     # the launch call itself
            big = np.argsort(st)[::-1][:4]
            log(f"[trace] {nsteps} steps: launch-to-launch ms largest {[(int(k), round(float(st[k]), 3)) for k in big]} "
                f"median {np.median(st):.3f}; launch call median {np.median(ln):.3f} max {ln.max():.3f} at {int(ln.argmax())}; "
                f"drain {1e3 * (tr[-1] - tr[2 * nsteps - 1]):.3f}")
        return kt, nk

    # Python's cyclic GC: a full collection traverses every host object -- the TOA tables and
    # flag lists of the whole PTA -- and took ~7 ms whenever it fell inside the timed steps
    # (a 20-step run: 0.40 or 0.73 ms per step by where it fell).  Collected once before the
    # warm-up and frozen (the objects alive now are never traversed again), no collection
    # until the timed steps end; a compiled host would have no such pause.  (Collected between
    # the warm-up and the timed steps instead, the device sat idle ~10 ms and the first timed
    # steps ran slower.)
    import gc
    gc.collect()
    gc.freeze()
    gc.disable()
    try:
        return _timed(sessions, steps, warmup, barrier, max_over_ranks, graph, gram_pass, pipes, run, step,
                      step_calls, replay)
    finally:
        gc.enable()
        gc.unfreeze()


def _timed(sessions, steps, warmup, barrier, max_over_ranks, graph, gram_pass, pipes, run, step, step_calls, replay):
    from pint_amd import _lib as L
    run(warmup * len(sessions), step, sessions)  # every pipeline warmed up
    if graph in (1, "1", "auto"):
        for s in sessions:
            s.set_timing_mask(0)
            for _ in range(L.NSLOT):  # one graph per pipeline slot
                s.capture(lambda: step_calls(s))
                s.check_step(s.step_end())
    # the candidates (launch mode, pipelines): fixed by the arguments, or timed on a short
    # trial each and the fastest kept
    modes = {"0": ["direct"], "1": ["hip-graph"], "auto": ["direct", "hip-graph"]}[str(graph)]
    npipe = list(range(1, len(sessions) + 1)) if pipes == "auto" else [min(int(pipes), len(sessions))]
    cands = [(m, p) for p in npipe for m in modes]
    if len(cands) > 1:
        # each candidate timed twice, the two passes in opposite orders (a drifting clock or a
        # host hiccup in one short run does not decide), the best of its two times kept
        ntry = max(20, min(50, steps // 2))
        times = {c: [] for c in cands}
        for order in (cands, cands[::-1]):
            for m, p in order:
                t0 = time.perf_counter()
                run(ntry, replay if m == "hip-graph" else step, sessions[:p])
                times[(m, p)].append(max_over_ranks(time.perf_counter() - t0))  # the same choice on every rank
        mode, p = min(cands, key=lambda c: min(times[c]))
    else:
        mode, p = cands[0]
    barrier()
    t0 = time.perf_counter()
    run(steps, replay if mode == "hip-graph" else step, sessions[:p])
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    # the Gram kernel's time: the same step with its events, after the timed region
    kt, nk = 0.0, 0
    s0 = sessions[0]
    if gram_pass:
        s0.set_timing_mask(1 << SLOT_GRAM)
        kt, nk = run(max(8 * GRAM_EVERY, steps // 2), step, [s0])  # (>= 8 sampled launches)
        s0.set_timing_mask(0)
    return dt, kt, nk, (lambda: step(s0)), mode, p


def c2_leg(batch, steps, warmup, world, barrier, max_over_ranks, max_pipes=1):
    """C2: B1855+09 NANOGrav 9-yr (4005 TOAs, DD, 72 DMX, 235 ECORR epochs,
    PLRedNoise; prepared here from its tim file) -- one GLSFitter.fit_toas(maxiter=1)
    end to end (host included, the reference's unit), and `batch` fits of it as one batched
    step (compact layout with the ECORR elimination, k_ecorr_dmx) on every rank."""
    import copy
    from pint_amd import GLSFitter
    from pint_amd.engine import Session, build_layout, pack_table
    from pint_amd.toa import get_model_and_toas
    g = os.path.join(ROOT, "tests", "golden")
    model, toas = get_model_and_toas(os.path.join(g, "B1855+09_NANOGrav_9yv1.gls.par"),
                                     os.path.join(g, "B1855+09_NANOGrav_9yv1.tim.gz"), ephem="builtin",
                                     include_bipm=False)
    out = {"workload": f"B1855+09 9-yr, {toas.ntoas} TOAs, {len(model.free_params)} free parameters (C2)"}
    dts = []
    for rep in range(4):  # the first fit is the warm-up
        f = GLSFitter(toas, copy.deepcopy(model))
        t0 = time.perf_counter()
        f.fit_toas(maxiter=1)
        dts.append(time.perf_counter() - t0)
    dt = float(np.median(dts[1:]))
    out["single_fit"] = {"metric": "GLSFitter fits/sec (maxiter=1, one fit, host included)",
                         "value": round(1.0 / dt, 3), "seconds": round(dt, 4), "chi2": float(f.resids.chi2)}
    ss = []
    for _ in range(max_pipes):  # (pipelines as the PTA leg: the fastest of 1..max_pipes on a trial)
        s = Session(device=int(os.environ.get("LOCAL_RANK", "0")))
        lay = s.add(build_layout(model, toas))
        s.set_instances([(lay, pack_table(lay, model))] * batch)
        ss.append(s)
    layout = ss[0].fit_layout(lay)
    dtb, kt, nk, _, launch, npipe = timed_steps(ss, steps, warmup, barrier, max_over_ranks, pipes="auto")
    for s in ss:
        s.close()
    out["batched"] = {"metric": f"GLS fits/sec, {batch} B1855 fits per batched step on each of {world} rank(s)",
                      "unit": "fits/s", "value": round(batch * world * steps / dtb, 1), "ms_per_step": round(dtb / steps * 1e3, 4),
                      "gram_ms": round(kt / max(1, nk), 4), "compact_layout": bool(layout[0]),
                      "gram_cols": layout[1], "dmx_cols": layout[2], "launch": launch, "pipelines": npipe}
    return out


def roofline(s, lays, kt_gram, step, args):
    """Roofline record of the dominant kernel (DESIGN.md §3 defines every count used here).

    k_gram_v (FP64 MFMA):
      alg_flops   useful flops of the normal matrix it forms, per TOA row: 2 x [(P+1)(P+2)/2
                  ([T|r]^T W [T|r], upper) + (P+1) R ([T|r]^T W F) + (P+2) (the row's DMX bin
                  entry against [T|r] and itself) + R (DMX x F)], P = compact timing columns,
                  R = 2 nred (F^T W F comes from the weighted trig sums, which depend on the
                  TOAs and sigma only: formed once per pulsar by k_trigw, not per launch);
      exec_flops  the MFMAs it issues, counted exactly as the kernel loops them: per N-split
                  ceil(rows / 64) chunks x 16 k-steps x NT tiles x 2048 flop (NT = the
                  [T|r|slots] x [T|r|slots|F] upper tiles less the all-slot (DD-only) tiles the
                  kernel skips; with the binned DMX x F tile (PINT_OPT_VBIN) the all-slot row
                  tiles go entirely and the binned tile comes); equals the PMC SQ_INSTS_MFMA x
                  2048 of the profile (profiles/pmc_gram_rNN.json).
    achieved = alg_flops / event time; exec_TFLOP/s beside it."""
    from pint_amd.pta import fit_cost  # noqa: F401
    nsplit = s.nsplit()
    alg = exe = 0.0
    for l in lays:
        vg, ns, kpv, r0 = s.vgram_layout(l)
        if not vg:
            continue
        vb = bool(vg & 2)  # binned DMX x F tile: the all-slot row tiles go, one binned tile comes
        n, R, nred = l.n, 2 * l.nred, l.nred
        P = r0
        alg += 2.0 * n * ((P + 1) * (P + 2) / 2 + (P + 1) * R + (P + 2) + R)
        ntr, ntc = (r0 + 1 + ns) // 16, kpv // 16
        nsk = ntr - (r0 + 1 + 15) // 16  # trailing all-slot row tiles: their DD-only tiles are skipped
        nt = 1 if vb else 0        # the binned tile
        for ti in range(ntr):      # as the kernel's loop skips them (gram_v_body)
            nt += sum(1 for tj in range(ti, ntc) if not (ti >= ntr - nsk and (tj < ntr or vb)))
        per = -(-n // nsplit)
        per = -(-per // 4) * 4
        chunks = sum(-(-max(0, min(n, (q + 1) * per) - min(n, q * per)) // 64) for q in range(nsplit))
        exe += chunks * 16.0 * nt * 2048.0
    # bytes the evaluation kernels move per TOA: inputs tdb (16) + freq (8) +
    # pos/vel/sun (72) + flags (4) + jump mask (8) + DMX ids (8) = 116 B; outputs phase hi/lo,
    # Taylor F, delay (32 B); the residual pass's first half fused into the evaluation (round
    # 6) reads the pulse-number offset and 1/sigma and writes the phase residual (24 B); with
    # the fit layout also the compact timing columns (8 P B) and the row's DMX value (8 B).
    # The residual pass left (k_resid2, post-fit, with the Woodbury trig tiles) reads the phase
    # residual, Taylor F, 1/sigma and the row's (cos, sin) of theta and 8 theta (56 B) and
    # writes the phase and time residuals (16 B)
    nrow = float(sum(l.n + 1 for l in lays))
    pc = [s.vgram_layout(l)[3] for l in lays]
    nbytes = {
        "k_eval": nrow * 172.0,
        "k_eval_M": float(sum((l.n + 1) * 172.0 + l.n * (8.0 * p + 8.0) for l, p in zip(lays, pc))),
        "k_resid": float(sum(l.n for l in lays)) * 72.0,
        # k_wsolve on the fused path (the dots come from k_resid2's tiles): per instance its
        # residual blocks' 16x16 tiles and chi2 partials, and the packed inverse factor of Sigma
        # -- a latency-bound per-instance forward substitution, not a streaming kernel
        "k_woodbury": float(sum(-(-l.n // 1024) * (256 + 3) * 8.0 + (2 * l.nred + 1) * (2 * l.nred + 2) / 2 * 8.0
                                for l in lays)),
    }
    # per-kernel breakdown: a separate instrumented pass (every timing slot's events on)
    s.set_timing_mask(0xFF)
    s.set_timing_every(1)
    kt = np.zeros(8)
    nprof = 3
    for _ in range(nprof):
        s.check_step(step())  # (one step in flight: its events alone on the streams)
        kt += s.timing()
    kt /= nprof
    names = ["k_eval", "k_resid", "gram_span", "k_solve", "k_eval_M", "k_woodbury", "k_gram", "k_greduce"]
    kms = {n: float(v) for n, v in zip(names, kt)}
    kms["k_gram"] = kt_gram  # the dominant kernel's time from the timed region itself
    ach = alg / (kt_gram * 1e-3) / 1e12 if kt_gram > 0 else None
    roof = {"kernel": "k_gram_v", "bound": "mfma",
            "achieved": round(ach, 3) if ach else None, "peak": MI355X_FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / MI355X_FP64_MFMA_PEAK_TFLOPS, 4) if ach else None,
            "traffic": pmc_value("pmc", "k_gram_v", "hbm_bytes", args)[0],
            "traffic_source": pmc_value("pmc", "k_gram_v", "hbm_bytes", args)[1],
            "alg_gflop_per_launch": round(alg / 1e9, 4), "exec_gflop_per_launch": round(exe / 1e9, 4),
            "exec_tflops": round(exe / (kt_gram * 1e-3) / 1e12, 3) if kt_gram > 0 else None,
            "exec_frac": round(exe / (kt_gram * 1e-3) / 1e12 / MI355X_FP64_MFMA_PEAK_TFLOPS, 4) if kt_gram > 0 else None,
            "pmc_exec_gflop_per_launch": pmc_value("pmc_gram", "k_gram_v", "mfma_gflop", args)[0],
            "pmc_mfma_busy_frac": pmc_value("pmc_gram", "k_gram_v", "mfma_busy_frac", args)[0],
            "pmc_valu_per_mfma": pmc_value("pmc_gram", "k_gram_v", "valu_per_mfma", args)[0],
            "pmc_source": pmc_value("pmc_gram", "k_gram_v", "mfma_gflop", args)[1],
            "kernel_ms": {n: round(v, 4) for n, v in kms.items()},
            "kernel_ms_source": ("k_gram: HIP events on its first/last dispatch packets, every "
                                 f"{GRAM_EVERY}th step of a pass after the timed region (averaged over those "
                                 f"launches; the timed steps carry no events); others: a separate "
                                 f"instrumented pass of {nprof} steps (gram_span = Gram + reduction)")}
    # what sets each one's time (the SQ counters of pmc_r06): the
    # evaluations' dependent FP64 chains at their occupancy, the residual pass's stream, the
    # Woodbury solve's per-instance substitution (its bytes are a few KB per pulsar)
    bound = {"k_eval": "fp64-latency", "k_eval_M": "fp64-latency", "k_resid": "hbm", "k_woodbury": "latency"}
    roof["per_kernel"] = {n: {"GB/s": round(b / (kms[n] * 1e-3) / 1e9, 1), "frac_hbm":
                              round(b / (kms[n] * 1e-3) / 1e9 / MI355X_HBM_PEAK_GBS, 4), "bound": bound.get(n)}
                          for n, b in nbytes.items() if kms.get(n, 0) > 0}
    gram_equiv = float(sum(2.0 * l.n * (l.K + 1.0) ** 2 for l in lays))
    roof["gram_full_equiv_tflops"] = round(gram_equiv / (kt_gram * 1e-3) / 1e12, 2) if kt_gram > 0 else None
    peaks = load_json("peaks_r03.json") or load_json("peaks_r02.json")
    if peaks:
        roof["measured_peaks"] = peaks
    return roof


def load_json(name):
    f = os.path.join(ROOT, "profiles", name)
    if os.path.exists(f):
        with open(f) as fh:
            return json.load(fh)
    return None


PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # newest first: the committed PMC summaries of this workload


def pmc_value(stem, kernel, key, args):
    """A per-launch PMC figure of `kernel` from the newest committed rocprofv3 summary
    (profiles/<stem>_rNN.json) of this same bench workload; HBM bytes = FETCH_SIZE x2 on
    gfx950 + WRITE_SIZE per MI355X_MICROARCH.md.  Returns (value, file) or (None, None)."""
    want = f"pta{args.npsr}x{args.ntoas // 1000}k"
    for r in PROFILE_ROUNDS:
        fname = f"{stem}_{r}.json"
        d = load_json(fname)
        if not d:
            continue
        if d.get("workload_key", d.get("workload", "").split(" ")[0]) != want:
            continue
        k = d.get("kernels", {}).get(kernel)
        if k is not None and k.get(key) is not None:
            return k.get(key), fname
    return None, None


def grid_leg(side, dist, barrier, max_over_ranks):
    """chi2 over a side x side (F0, F1) grid, WLSFitter per point (gridutils.py:166 parallel
    semantics), points sharded over ranks; the median of three full grids."""
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
    for _ in range(2):  # warm-up: the TOAs uploaded, batch buffers allocated (the 2nd grid was still slow)
        grid_chisq(f, ("F0", "F1"), (g0, g1))
    dts = []
    for _ in range(3):
        barrier()
        t0 = time.perf_counter()
        chi2, _ = grid_chisq(f, ("F0", "F1"), (g0, g1))
        barrier()
        dts.append(max_over_ranks(time.perf_counter() - t0))
    dt = float(np.median(dts))
    # per-kernel device time of one more grid (every timing slot's HIP events on, the grid's
    # points as one batch on one session = one fit step; after the timed grids, which carry
    # no events and run on gridutils.GRID_PIPES concurrent sessions)
    from pint_amd import gridutils
    npipe = gridutils.GRID_PIPES
    gridutils.GRID_PIPES = 1
    try:
        gs, glay = gridutils._GRID["cur"][1][0]
        gs.set_timing_mask(0xFF)
        grid_chisq(f, ("F0", "F1"), (g0, g1))
        kt = gs.timing()
        gs.set_timing_mask(0)
    finally:
        gridutils.GRID_PIPES = npipe
    roof = grid_roofline(kt, glay, side * side, dt)
    out = {"metric": "chi2-grid points/sec", "value": round(side * side / dt, 1), "unit": "points/s",
           "workload": f"NGC6440E (62 TOAs) {side}x{side} (F0,F1) WLSFitter", "seconds": round(dt, 4),
           "seconds_all": [round(x, 4) for x in dts], "timing": "median of 3 grids after 2 warm-up grids",
           "pipelines": gridutils.GRID_PIPES if side * side >= 2 * gridutils.GRID_PIPE_MIN else 1,
           "chi2_min": float(np.nanmin(chi2)), "roofline": roof}
    if dist is None:
        out["predicted_strong"] = grid_emulate(f, g0, g1, side, dt)
    return out


def grid_emulate(f, g0, g1, side, dt1, worlds=(2, 4, 8)):
    """Predicted strong scaling of the grid leg on this one GPU: for each world size N, the
    contiguous blocks of the flattened meshgrid that ranks 0 and N-1 own in an N-rank run
    (gridutils.shard_range; every other rank's block equals rank 0's) are fitted alone, the
    median of 3 after a warm-up each; the predicted N-GPU grid time is the slower block's."""
    from pint_amd import gridutils
    from pint_amd.gridutils import grid_chisq
    npts = side * side
    out = {"method": ("ranks 0 and N-1's contiguous point blocks (gridutils.shard_range) each fitted alone on "
                      "this GPU, median of 3 after a warm-up; predicted value = points / the slower block's time"),
           "n1": {"value": round(npts / dt1, 1), "seconds": round(dt1, 6)}}
    for nw in worlds:
        per = []
        for r in sorted({0, nw - 1}):
            gridutils._EMULATE_SHARD = (r, nw)
            try:
                grid_chisq(f, ("F0", "F1"), (g0, g1))  # warm-up (the block's batch set up)
                reps = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    grid_chisq(f, ("F0", "F1"), (g0, g1))
                    reps.append(time.perf_counter() - t0)
            finally:
                gridutils._EMULATE_SHARD = None
            per.append(float(np.median(reps)))
        mx = max(per)
        out[f"n{nw}"] = {"value": round(npts / mx, 1), "seconds": round(mx, 6),
                         "points_per_rank": gridutils.shard_range(npts, 0, nw)[0],
                         "speedup_vs_n1": round(dt1 / mx, 3)}
        log(f"[grid emulate {nw}] blocks {[round(p * 1e3, 3) for p in per]} ms -> {npts / mx:.0f} points/s")
    return out


def grid_roofline(kt, lay, npts, dt):
    """Roofline record of the grid step's dominant kernel.

    The grid's points share one pulsar's TOAs, so a launch's algorithmic bytes are the TOA
    inputs once ((n+1) x 116 B, then L2-resident) plus every point's own outputs: with M
    (k_eval_M) (n+1) x 32 B (phase hi/lo, Taylor F, delay) + n x 8 K B (the design matrix);
    without M the 32 B rows; the residual passes 80 B per point row; the Gram 8 (K+1) B per
    row read.  None of them reaches HBM speed: the evaluation is bound by its FP64 VALU issue
    (pmc_valu_busy from the committed PMC summary of this grid, profiles/pmc_grid_rNN.json)."""
    names = ["k_eval", "k_resid", "gram_span", "k_solve", "k_eval_M", "k_woodbury", "k_gram", "k_greduce"]
    kms = {n: round(float(v), 4) for n, v in zip(names, kt)}
    n, K = lay.n, lay.K
    nbytes = {"k_eval_M": (n + 1) * 116.0 + npts * ((n + 1) * 32.0 + n * 8.0 * K),
              "k_eval": (n + 1) * 116.0 + npts * (n + 1) * 32.0,
              "k_resid": npts * n * 80.0,
              "k_gram": npts * n * 8.0 * (K + 1)}
    dom = max(nbytes, key=lambda k: kms.get(k, 0.0))
    t = kms[dom] * 1e-3
    ach = nbytes[dom] / t / 1e9 if t > 0 else None
    traffic, src = pmc_grid(dom, "hbm_bytes")
    valu, _ = pmc_grid(dom, "valu_busy_frac")
    return {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1) if ach else None, "peak": MI355X_HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / MI355X_HBM_PEAK_GBS, 4) if ach else None,
            "traffic": traffic, "traffic_source": src, "alg_bytes_per_launch": nbytes[dom],
            "pmc_valu_busy_frac": valu,
            "per_kernel": {k: {"GB/s": round(b / (kms[k] * 1e-3) / 1e9, 1)} for k, b in nbytes.items() if kms.get(k, 0) > 0},
            "kernel_ms": kms, "grid_ms": round(dt * 1e3, 3), "points": npts, "rows_per_point": n, "K": K,
            "kernel_ms_source": "HIP events of every timing slot on one more grid after the timed grids"}


def pmc_grid(kernel, key):
    """A per-launch PMC figure of the NGC6440E 256x256 grid's kernel from the newest
    profiles/pmc_grid_rNN.json (scripts/gpu_prof.sh + scripts/pmc_grid_summary.py)."""
    for r in PROFILE_ROUNDS:
        d = load_json(f"pmc_grid_{r}.json")
        k = (d or {}).get("kernels", {}).get(kernel)
        if k is not None and k.get(key) is not None:
            return k[key], f"pmc_grid_{r}.json"
    return None, None


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
    frozen = model.find_empty_masks(toas, freeze=True)
    return model, toas, frozen


def j0740_legs(side, dist, barrier, max_over_ranks):
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
    dts = []
    for rep in range(4):  # the first fit is the warm-up (library load, first-call allocations)
        f = DownhillGLSFitter(toas, copy.deepcopy(model))
        barrier()
        t0 = time.perf_counter()
        try:
            f.fit_toas(maxiter=10)
            conv = True
        except MaxiterReached:
            conv = False
        dts.append(time.perf_counter() - t0)
    dt = float(np.median(dts[1:]))  # one fit is ~30-40 ms of mostly host work: the median of 3
    out["downhill_gls"] = {"metric": "DownhillGLSFitter fits/sec (maxiter=10)", "value": round(1.0 / dt, 3),
                           "seconds": round(dt, 4), "seconds_all": [round(x, 4) for x in dts[1:]],
                           "converged": conv, "chi2": float(f.resids.chi2)}
    g = GLSFitter(toas, copy.deepcopy(model))
    g.fit_toas(maxiter=1)
    m2 = np.linspace(0.2, 0.3, side)
    sini = np.sin(np.deg2rad(np.linspace(86.25, 88.5, side)))
    grid_chisq(g, ("M2", "SINI"), (m2, sini))  # warm-up (first-touch of the batch buffers)
    barrier()
    t0 = time.perf_counter()
    chi2, _ = grid_chisq(g, ("M2", "SINI"), (m2, sini))
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    out["grid_m2_sini"] = {"metric": "chi2-grid points/sec", "value": round(side * side / dt, 1),
                           "unit": "points/s", "workload": f"J0740 50k TOAs {side}x{side} (M2,SINI) GLSFitter",
                           "seconds": round(dt, 3), "chi2_min": float(np.nanmin(chi2))}
    return out


# ---- CPU baseline: the oracle (numpy longdouble restatement) on the host's cores ---------
_CPU_ITEMS = None


def _cpu_init(items, root):
    global _CPU_ITEMS
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)  # one BLAS thread per worker process
    except Exception:
        pass
    _CPU_ITEMS = items


def _cpu_fits(args):
    """Worker: GLS fits (maxiter=1 + post-fit chi2) of item k for `budget` seconds."""
    k, budget = args
    import pint_oracle as O
    model, toas = _CPU_ITEMS[k % len(_CPU_ITEMS)]
    t0 = time.perf_counter()
    n = 0
    while True:
        O.gls_fit_from_product_inputs(model, toas)
        n += 1
        if time.perf_counter() - t0 > budget:
            return n


def _cpu_grid(args):
    """Worker: WLS fits of NGC6440E grid points (F0, F1 frozen at the point) for `budget` s."""
    k, budget = args
    import pint_oracle as O
    om, ot, f0s, f1s = _CPU_ITEMS
    t0 = time.perf_counter()
    n = 0
    while True:
        j = (k * 7919 + n) % len(f0s)
        O.grid_chisq(om, ot, ("F0", "F1"), ([f0s[j]], [f1s[j]]), gls=False)
        n += 1
        if time.perf_counter() - t0 > budget:
            return n


def host_cores():
    """The job's CPU share: the cgroup v2 quota (cpu.max "quota period") when one is set,
    capped by the affinity mask; otherwise the affinity mask.  Returns (cores, note)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    note = f"affinity {aff}, os.cpu_count {os.cpu_count()}"
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(f).read().split()
        except OSError:
            continue
        if f.endswith("cpu.max"):
            if txt and txt[0] != "max":
                q = int(txt[0]) / int(txt[1])
                note += f", cgroup cpu.max {txt[0]} {txt[1]} = {q:g} cores"
                return max(1, min(aff, int(q + 0.5))), note
            note += ", cgroup cpu.max: no quota"
        else:
            q = int(txt[0])
            if q > 0:
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                note += f", cfs quota {q}/{per}"
                return max(1, min(aff, int(q / per + 0.5))), note
        break
    return aff, note


def cpu_baseline(items):
    """The oracle (oracle/pint_oracle.py, numpy longdouble) timed on this host on bounded
    samples, one process per core of the job's CPU share (host_cores: cgroup quota, else affinity):
    GLS fits of the PTA's own 10k-TOA pulsars, and WLS grid points of NGC6440E -- the GPU
    workloads' units.  The reference's own CPU rates (measured in the build container; the
    reference cannot travel to the GPU box) are attached from bench/reference_cpu.json."""
    import multiprocessing as mp
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pint_oracle as O  # noqa: F401
    except Exception as e:  # oracle missing: report, never fall back
        return {"value": None, "error": repr(e)}
    ncores, quota_note = host_cores()
    nproc = max(1, ncores)
    ctx = mp.get_context("spawn")  # never fork a process that holds a GPU context
    # one BLAS/OpenMP thread per worker (the box exports OMP_NUM_THREADS=16: 16 workers x 16
    # threads would oversubscribe the job's cores); the spawned workers inherit this
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        return _cpu_baseline_pools(items, ctx, nproc, quota_note)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _cpu_baseline_pools(items, ctx, nproc, quota_note):
    budget = 10.0
    with ctx.Pool(nproc, initializer=_cpu_init, initargs=(items[:nproc], ROOT)) as pool:
        t0 = time.perf_counter()
        counts = pool.map(_cpu_fits, [(k, budget) for k in range(nproc)])
        dt = time.perf_counter() - t0
    fits = sum(counts)
    out = {"value": round(fits / dt, 4), "unit": "fits/s", "cores": nproc, "kind": "port",
           "sample": f"{fits} GLS fits (maxiter=1 + post-fit GLS chi2) of {min(nproc, len(items))} of the PTA's 10k-TOA pulsars, "
                     f"one oracle process per core (numpy longdouble, 1 BLAS thread each), {dt:.1f} s wall; "
                     f"job CPU share: {quota_note}"}
    # grid points: NGC6440E (F0, F1) WLS fits, the grid leg's unit
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import load
    import pint_oracle as O
    model, toas, z, _ = load("ngc6440e")
    om, ot = O.from_product_model(model), O.toas_from_product(toas)
    g0 = z["grid_F0_hi"].astype(np.longdouble) + z["grid_F0_lo"]
    g1 = z["grid_F1_hi"].astype(np.longdouble) + z["grid_F1_lo"]
    f0s, f1s = [x.ravel() for x in np.meshgrid(g0, g1)]
    gb = 5.0
    with ctx.Pool(nproc, initializer=_cpu_init, initargs=((om, ot, f0s, f1s), ROOT)) as pool:
        t0 = time.perf_counter()
        counts = pool.map(_cpu_grid, [(k, gb) for k in range(nproc)])
        dt = time.perf_counter() - t0
    out["grid"] = {"value": round(sum(counts) / dt, 2), "unit": "points/s", "cores": nproc,
                   "sample": f"{sum(counts)} NGC6440E (F0,F1) WLS grid points, {nproc} processes, {dt:.1f} s"}
    ref = os.path.join(ROOT, "bench", "reference_cpu.json")
    if os.path.exists(ref):
        with open(ref) as fh:
            out["reference_container"] = json.load(fh)
    return out


if __name__ == "__main__":
    main()
