"""Gram timing events with PINT_OPT_TIMING_EVERY: print slot 6 after each pipelined step."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pint_amd import simulation as sim  # noqa: E402
from pint_amd.engine import Session, build_layout, pack_table  # noqa: E402

items = sim.make_pta(ntoas=10000, indices=list(range(68)))
s = Session()
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
s.save_tables()
s.set_timing_mask(1 << 6)
for k in range(3):  # synchronous, no sampling option touched
    s.restore_tables()
    s.eval(want_M=Session.FIT)
    s.fit_step(1)
    s.check()
    print(f"sync step {k}: gram {s.timing()[6] * 1e3:8.1f} us, all {np.round(s.timing() * 1e3, 1)}")
s.set_timing_mask(0xFF)
s.restore_tables()
s.eval(want_M=Session.FIT)
s.fit_step(1)
s.check()
print(f"sync mask ff: {np.round(s.timing() * 1e3, 1)}")
s.set_lazy(True)
for every in (1, 4):
    s.set_timing_mask(1 << 6)
    s.set_timing_every(every)
    prev = None
    t0 = time.perf_counter()
    for k in range(12):
        s.restore_tables()
        s.eval(want_M=Session.FIT)
        s.fit_step(1)
        s.read_step()
        s.noise_resids()
        s.apply_step_uniform(1.0)
        s.eval(want_M=False)
        s.chi2_gls()
        cur = s.step_end()
        if prev is not None:
            s.check_step(prev)
            print(f"every {every} step {k - 1}: gram {s.timing()[6] * 1e3:8.1f} us")
        prev = cur
    s.check_step(prev)
    print(f"every {every}: {(time.perf_counter() - t0) / 12 * 1e3:.3f} ms/step")
s.close()
