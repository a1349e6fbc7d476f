"""k_solve_dmx phase timestamps of workgroup 0 (s_memrealtime, 100 MHz; pint_debug_read(.., 4)):
    python scripts/diag/ts_probe.py NPSR [apply]
apply: the bench's step (lazy, restore, fused apply).  Only phases whose timestamps were
written by this launch (inside its [start, end] span, increasing) are printed; a phase that
did not run (e.g. the refinement when the condition estimate is below its threshold) is
reported as not run instead of as a difference of stale timestamps."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from pint_amd import _lib as L
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 68
APPLY = len(sys.argv) > 2 and sys.argv[2] == "apply"
items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)))
s = Session(0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
if APPLY:
    s.save_tables()
    s.set_lazy(True)


def span(out, a, b):
    """b - a in us when both stamps belong to this launch, else None."""
    t0, t1 = out[0], out[7]
    if not (t0 <= out[a] <= t1 and t0 <= out[b] <= t1 and out[b] >= out[a] and (a == 0 or out[a] > 0)):
        return None
    return out[b] - out[a]


def fmt(v):
    return "  n/a " if v is None else f"{v:6.2f}"


for it in range(4):
    s.L.pint_debug_read(s.ctx, 6, None)  # reset the stamps
    if APPLY:
        s.restore_tables()
        s.eval(want_M=Session.FIT)
        s.fit_step_apply(1, 1.0)
        s.read_step()
        s.check()
    else:
        s.eval(want_M=Session.FIT)
        s.fit_step(1)
    out = np.zeros(32)
    s.L.pint_debug_read(s.ctx, 4, L.ptr(out))
    out = out.astype(np.float64)
    if it == 0:
        continue  # first launch: code-object load, cold caches
    names = ["build (or k_schur's load)", "S-=UU'+b'", "chol+inv", "y", "x+refine+steps", "export", "tail"]
    print("step", it, "wg0 us", fmt(span(out, 0, 7)),
          " | ".join(f"{n} {fmt(span(out, k, k + 1))}" for k, n in enumerate(names)))
    print("   diag factor 0 %s | panel 0 %s | trailing 0 %s | inverse rows %s" % (
        fmt(span(out, 9, 10)), fmt(span(out, 11, 12)), fmt(span(out, 12, 13)), fmt(span(out, 14, 16))))
    r = span(out, 17, 21)
    print("   refinement", "not run" if r is None else f"{r:.2f} us",
          "| steps->setup %s setup %s" % (fmt(span(out, 5, 22)), fmt(span(out, 22, 23))))
