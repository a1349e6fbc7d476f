"""Per-workgroup timeline of one pipelined PTA fit step (the bench's step) at NPSR pulsars:
every instrumented kernel's workgroups (WgTimer: first stamp of thread 0, last wave's exit)
-> per kernel the dispatch spread, the workgroup durations and the span, relative to the
step's first stamp (us).  Tells a kernel's launch ramp from its longest workgroup.

    python3 scripts/diag/wg_timeline.py [NPSR] [STEPS]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from pint_amd import _lib as L
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

NAMES = ["eval", "gram_v", "greduce", "schur", "solve_dmx", "resid1", "resid2", "wsolve", "cov_dmx", "noise_red",
         "export", "other"]
KB = 2048
NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 9
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5

items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)))
s = Session(0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
s.save_tables()
s.set_lazy(True)
s.set_timing_mask(0)
for _ in range(10):  # warm-up
    s.check_step(s.fit_step_enqueue(restore=True, lam=1.0)[0])
buf = np.zeros(len(NAMES) * KB * 2)
rows = {n: [] for n in NAMES}
spans = []
for it in range(STEPS):
    on = np.ones(1)
    s.L.pint_debug_read(s.ctx, 8, L.ptr(on))
    s.check_step(s.fit_step_enqueue(restore=True, lam=1.0)[0])
    s.L.pint_debug_read(s.ctx, 7, L.ptr(buf))
    t = buf.reshape(len(NAMES), KB, 2)
    used = t[:, :, 0] > 0
    t0 = t[:, :, 0][used].min()
    spans.append((t[:, :, 1][used].max() - t0) * 0.01)
    for k, n in enumerate(NAMES):
        u = used[k]
        if not u.any():
            continue
        st = (t[k, u, 0] - t0) * 0.01
        en = (t[k, u, 1] - t0) * 0.01
        du = en - st
        rows[n].append((u.sum(), st.min(), st.max(), np.median(du), du.max(), en.max()))
    off = np.zeros(1)
    s.L.pint_debug_read(s.ctx, 8, L.ptr(off))
print(f"{NPSR} pulsars, {STEPS} steps; step span (first stamp to last exit) median {np.median(spans):.1f} us")
print(f"{'kernel':10s} {'WGs':>5s} {'start':>7s} {'last st':>7s} {'med dur':>7s} {'max dur':>7s} {'end':>7s}  (us)")
order = sorted([n for n in NAMES if rows[n]], key=lambda n: np.median([r[1] for r in rows[n]]))
for n in order:
    r = np.median(np.array(rows[n]), axis=0)
    print(f"{n:10s} {int(r[0]):5d} {r[1]:7.1f} {r[2]:7.1f} {r[3]:7.1f} {r[4]:7.1f} {r[5]:7.1f}")
s.close()
