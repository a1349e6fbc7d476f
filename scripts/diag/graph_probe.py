"""Small-batch step: host enqueue vs device time, direct launches vs a HIP-graph replay.
    python scripts/diag/graph_probe.py NPSR [STEPS]
Prints ms/step for (1) the bench's pipelined direct step, (2) direct steps enqueued back to
back with one synchronisation at the end (host-enqueue bound when the host is slower),
(3) the same step captured once into a HIP graph and replayed back to back, (4) graph
replays synchronised every step (latency of one step)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pint_amd import simulation as sim  # noqa: E402
from pint_amd.engine import Session, build_layout, pack_table  # noqa: E402

npsr = int(sys.argv[1]) if len(sys.argv) > 1 else 9
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
items = sim.make_pta(ntoas=10000, indices=list(range(npsr)))
s = Session(0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
s.save_tables()
s.set_lazy(True)
s.set_timing_mask(0)


def step():
    s.restore_tables()
    s.eval(want_M=Session.FIT)
    s.fit_step(1)
    out = s.read_step()
    nz = s.noise_resids()
    s.apply_step_uniform(1.0)
    s.eval(want_M=False)
    return out, nz, s.chi2_gls()


def pipelined(n):
    prev = None
    for _ in range(n):
        step()
        cur = s.step_end()
        if prev is not None:
            s.check_step(prev)
        prev = cur
    s.check_step(prev)


pipelined(20)
t0 = time.perf_counter()
pipelined(K)
t_pipe = (time.perf_counter() - t0) / K

# host enqueue alone: steps enqueued back to back (one slot), timed without the final sync
for _ in range(10):
    step()
s.check()
t0 = time.perf_counter()
for _ in range(K):
    step()
t_enq = (time.perf_counter() - t0) / K
s.check()
t_back = (time.perf_counter() - t0) / K

ref = step()
s.check()
c2_direct = np.array(ref[2]).copy()
cap = s.capture(step)
for _ in range(10):
    s.replay()
s.check()
t0 = time.perf_counter()
for _ in range(K):
    s.replay()
t_genq = (time.perf_counter() - t0) / K
s.check()
t_graph = (time.perf_counter() - t0) / K
assert np.array_equal(np.array(cap[2]), c2_direct), "graph replay differs from the direct step"
t0 = time.perf_counter()
for _ in range(K // 4):
    s.replay()
    s.check()
t_glat = (time.perf_counter() - t0) / (K // 4)
print(f"npsr {npsr}: pipelined direct {t_pipe * 1e3:.4f} ms/step | direct back-to-back {t_back * 1e3:.4f} "
      f"(host enqueue {t_enq * 1e3:.4f}) | graph back-to-back {t_graph * 1e3:.4f} (enqueue {t_genq * 1e3:.4f}) | "
      f"graph synchronised {t_glat * 1e3:.4f} ms/step")
s.close()
