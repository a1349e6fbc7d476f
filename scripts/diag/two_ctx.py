"""Two fits in flight: the bench step on one Session against the same step alternated over
two Sessions (two contexts, each with its own streams and buffers, the same 68-pulsar PTA),
so the low-occupancy kernels of one (solve, reductions, set-up) can share the GPU with the
other's evaluation and Gram.  Prints ms per fit step for 1 and 2 contexts; env
GPU_MAX_HW_QUEUES is reported (each context uses three streams)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pint_amd import simulation as sim  # noqa: E402
from pint_amd.engine import Session, build_layout, pack_table  # noqa: E402

items = sim.make_pta(ntoas=10000, indices=list(range(68)))


def make():
    s = Session()
    lays = [s.add(build_layout(m, t)) for m, t in items]
    s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
    s.save_tables()
    s.set_lazy(True)
    s.set_timing_mask(0)
    return s


def step(s):
    s.restore_tables()
    s.eval(want_M=Session.FIT)
    s.fit_step(1)
    s.read_step()
    s.noise_resids()
    s.apply_step_uniform(1.0)
    s.eval(want_M=False)
    s.chi2_gls()


def run(sessions, nsteps):
    prev = [None] * len(sessions)
    t0 = time.perf_counter()
    for k in range(nsteps):
        j = k % len(sessions)
        s = sessions[j]
        step(s)
        cur = s.step_end()
        if prev[j] is not None:
            s.check_step(prev[j])
        prev[j] = cur
    for s, p in zip(sessions, prev):
        if p is not None:
            s.check_step(p)
    return (time.perf_counter() - t0) / nsteps * 1e3


print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))
a = make()
run([a], 20)
print(f"1 context : {run([a], 100):.4f} ms/step")
b = make()
run([a, b], 20)
print(f"2 contexts: {run([a, b], 100):.4f} ms/step")
print(f"1 context : {run([a], 100):.4f} ms/step")
a.close()
b.close()
