"""(experiment) The bench's 68 x 10k PTA fit step as one batch on one stream against two
34-pulsar batches on two contexts (two HIP streams) driven alternately: do the latency-bound
stretches of one batch (solve, prep/apply, Woodbury solve) overlap the other's full-chip
kernels?  Prints ms per 68-pulsar step for both."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from pint_amd import simulation as sim  # noqa: E402
from pint_amd.engine import Session, build_layout, pack_table  # noqa: E402

models = [sim.pta_model(i) for i in range(68)]
items = sim.make_pta(ntoas=10000, indices=list(range(68)), models=models)


def make(sub):
    s = Session(device=0)
    lays = [s.add(build_layout(m, t)) for m, t in sub]
    tabs = [pack_table(l, m) for l, (m, _) in zip(lays, sub)]
    s.set_instances(list(zip(lays, tabs)))
    s.set_lazy(True)
    s.set_timing_mask(0)
    return s, np.concatenate(tabs), np.ones(len(lays))


def step(ctx):
    s, flat, ones = ctx
    s.set_tables(flat)
    s.eval(want_M=Session.FIT)
    s.fit_step(1)
    s.read_step()
    s.apply_step(ones)
    s.eval(want_M=False)
    s.chi2_gls()


def timed(ctxs, nsteps):
    prev = [None] * len(ctxs)
    t0 = time.perf_counter()
    for _ in range(nsteps):
        for k, c in enumerate(ctxs):
            step(c)
            cur = c[0].step_end()
            if prev[k] is not None:
                c[0].check_step(prev[k])
            prev[k] = cur
    for k, c in enumerate(ctxs):
        if prev[k] is not None:
            c[0].check_step(prev[k])
    return (time.perf_counter() - t0) / nsteps * 1e3


one = [make(items)]
timed(one, 3)
print(f"one batch of 68: {timed(one, 30):.4f} ms/step", flush=True)
one[0][0].close()
# split by LPT-like alternation so both halves carry the same model mix
two = [make(items[0::2]), make(items[1::2])]
timed(two, 3)
print(f"two batches of 34 on two streams: {timed(two, 30):.4f} ms per 68-pulsar step", flush=True)
for c in two:
    c[0].close()
