"""Throughput of the bench's PTA step with P independent pipelines (sessions, each its own
streams and buffers) fed round-robin, against one: NPSR pulsars, STEPS steps per run.

    python3 scripts/diag/two_pipes.py [NPSR] [STEPS] [P]
"""
import gc
import os
import sys
import time
from collections import deque

import numpy as np

sys.path.insert(0, os.getcwd())
from pint_amd import _lib as L
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 9
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
P = int(sys.argv[3]) if len(sys.argv) > 3 else 2

items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)))
ss = []
for _ in range(P):
    s = Session(0)
    lays = [s.add(build_layout(m, t)) for m, t in items]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
    s.save_tables()
    s.set_lazy(True)
    s.set_timing_mask(0)
    ss.append(s)


def run(sessions, n):
    pend = [deque() for _ in sessions]
    t0 = time.perf_counter()
    for i in range(n):
        k = i % len(sessions)
        s = sessions[k]
        if len(pend[k]) >= L.NSLOT:
            s.check_step(pend[k].popleft())
        pend[k].append(s.fit_step_enqueue(restore=True, lam=1.0)[0])
    for k, s in enumerate(sessions):
        while pend[k]:
            s.check_step(pend[k].popleft())
    return time.perf_counter() - t0


gc.collect()
gc.freeze()
gc.disable()
for p in range(1, P + 1):
    run(ss[:p], 20)
    r = [run(ss[:p], STEPS) / STEPS * 1e3 for _ in range(3)]
    print(f"{NPSR} pulsars, {p} pipeline(s): ms per step {np.median(r):.4f} (runs {[round(x, 4) for x in r]}) "
          f"-> {NPSR / np.median(r) * 1e3:.0f} fits/s")
for s in ss:
    s.close()
