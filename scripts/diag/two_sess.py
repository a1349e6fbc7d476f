"""Experiment: the 68-pulsar PTA step as two half-batches on two contexts (streams), their
steps enqueued alternately, so one half's narrow kernels (solve, reductions) overlap the
other's wide ones (evaluation, Gram).  Prints ms per whole-PTA step for 1 and 2 contexts.

Result (round 5, one MI355X): 1 context 0.47-0.48 ms per step, 2 contexts 0.74-0.84, 3
contexts 0.69 -- the contexts' streams share the process's 4 hardware queues and their
steps serialise with extra gaps; dropped."""
import os
import sys
import time
from collections import deque

import numpy as np

sys.path.insert(0, os.getcwd())
from pint_amd import _lib as L
L.lib()
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table
from pint_amd.pta import fit_cost, lpt_shard

NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 68
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
models = [sim.pta_model(i) for i in range(NPSR)]
items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)), models=models)
costs = [fit_cost(m, n=10000) for m in models]


def sessions(nsplit):
    out = []
    for sh in lpt_shard(costs, nsplit):
        s = Session(0)
        sub = [items[i] for i in sh]
        lays = [s.add(build_layout(m, t)) for m, t in sub]
        s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, sub)])
        s.save_tables()
        s.set_lazy(True)
        out.append(s)
    return out


def run(ss, nsteps):
    pend = [deque() for _ in ss]
    for _ in range(nsteps):
        for s, p in zip(ss, pend):
            if len(p) >= L.NSLOT:
                s.check_step(p.popleft())
            p.append(s.fit_step_enqueue(restore=True)[0])
    for s, p in zip(ss, pend):
        while p:
            s.check_step(p.popleft())


for nsplit in (1, 2, 3, 1, 2):
    ss = sessions(nsplit)
    run(ss, 10)
    t0 = time.perf_counter()
    run(ss, STEPS)
    dt = (time.perf_counter() - t0) / STEPS
    print(f"{nsplit} context(s): {dt * 1e3:.4f} ms per {NPSR}-pulsar step ({NPSR / dt:.0f} fits/s)", flush=True)
    for s in ss:
        s.close()
