"""Phase split of the evaluation blocks at NPSR pulsars: per workgroup, the LDS staging
prologue (first stamp -> after its barrier), the rows' evaluation (-> last wave's row end)
and the rest (the fused residual pass, exit), for the fit-layout evaluation (design matrix)
and for the phase-only one (us, medians over workgroups and repeats).

    python3 scripts/diag/eval_phases.py [NPSR] [REPS]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from pint_amd import _lib as L
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

KB = 2048
NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 68
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5

items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)))
s = Session(0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
s.save_tables()
s.set_lazy(True)
s.set_timing_mask(0)
for _ in range(5):
    s.check_step(s.fit_step_enqueue(restore=True, lam=1.0)[0])
t = np.zeros(12 * KB * 2)
p = np.zeros(KB * 2)
for label, mode in (("fit layout (M)", s.FIT), ("phases only", False)):
    res = []
    for _ in range(REPS):
        s.L.pint_debug_read(s.ctx, 8, L.ptr(np.ones(1)))
        s.eval(mode)
        s.L.pint_debug_read(s.ctx, 7, L.ptr(t))
        s.L.pint_debug_read(s.ctx, 9, L.ptr(p))
        st, en = t[0:KB * 2:2], t[1:KB * 2:2]
        pe, re = p[0::2], p[1::2]
        u = (st > 0) & (pe > 0) & (re > 0)
        t0 = st[u].min()
        res.append([u.sum(), np.median(pe[u] - st[u]) * 0.01, np.median(re[u] - pe[u]) * 0.01,
                    np.median(en[u] - re[u]) * 0.01, np.median(en[u] - st[u]) * 0.01,
                    (st[u].max() - t0) * 0.01, (en[u].max() - t0) * 0.01])
    r = np.median(np.array(res), axis=0)
    print(f"{label:15s} WGs {int(r[0]):5d}  prologue {r[1]:6.2f}  rows {r[2]:6.2f}  tail {r[3]:6.2f}  "
          f"WG {r[4]:6.2f}  last start {r[5]:6.1f}  span {r[6]:6.1f}  (us, first {KB} WGs)")
s.L.pint_debug_read(s.ctx, 8, L.ptr(np.zeros(1)))
s.close()
