"""Evaluation kernel time per binary model: the bench PTA's isolated, ELL1 and DD pulsars
each as a batch of its own, eval with the fit-layout design matrix and eval without,
timed with the library's HIP events (timing slots 0 = eval, 4 = eval with M)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pint_amd import simulation as sim  # noqa: E402
from pint_amd.engine import Session, build_layout, pack_table  # noqa: E402

items = sim.make_pta(ntoas=10000, indices=list(range(68)))
groups = {"iso": [], "ELL1": [], "DD": []}
for i, it in enumerate(items):
    groups[sim.pta_kind(i) or "iso"].append(it)
groups["all"] = items
for name, its in groups.items():
    s = Session()
    lays = [s.add(build_layout(m, t)) for m, t in its]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, its)])
    s.set_timing_mask(0xFF)
    tm, t0 = [], []
    for rep in range(6):
        s.eval(want_M=Session.FIT)
        s.check()
        tm.append(s.timing()[4])
        s.eval(want_M=False)
        s.check()
        t0.append(s.timing()[0])
    n = sum(t.ntoas for _, t in its)
    em, e0 = np.median(tm[1:]), np.median(t0[1:])
    print(f"{name:5s} {len(its):3d} psrs {n:7d} rows: eval+M {em * 1e3:7.1f} us ({em * 1e6 / n:6.2f} ns/row)  "
          f"eval {e0 * 1e3:7.1f} us ({e0 * 1e6 / n:6.2f} ns/row)")
    s.close()
