"""Throughput of the bench step with the 68-pulsar PTA split over S sessions (own HIP
streams and buffers), each pipelined two deep; the sessions' kernels overlap on the GPU."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pint_amd.engine import Session, build_layout, pack_table
from pint_amd import simulation as sim
from pint_amd.timing_model import get_model
npsr = 68
specs = []
for i in range(npsr):
    kind = "ELL1" if i % 6 in (1, 4) else ("DD" if i % 6 == 2 else "")
    m = get_model(sim.pta_par(i, kind))
    specs.append(dict(model=m, start=53000, end=56652, ntoas=10000, freq=[800, 1200, 1600, 2000],
                      obs="geocenter", error_us=0.5, add_noise=True, add_correlated_noise=True, seed=i))
toas = sim.make_fake_toas_batch(specs)
for S in [1, 2, 3, 4]:
    sess = []
    for k in range(S):
        idx = list(range(k, npsr, S))
        s = Session()
        lays = [s.add(build_layout(specs[i]["model"], toas[i])) for i in idx]
        tabs = [pack_table(l, specs[i]["model"]) for l, i in zip(lays, idx)]
        s.set_instances(list(zip(lays, tabs)))
        s.set_lazy(True)
        s.set_timing_mask(0)
        sess.append((s, np.concatenate(tabs), np.ones(len(idx))))

    def step(s, flat, ones):
        s.set_tables(flat)
        s.eval(want_M=Session.FIT)
        s.fit_step(1)
        s.read_step()
        s.apply_step(ones)
        s.eval(want_M=False)
        s.chi2_gls()

    def run(n):
        prev = [None] * S
        for _ in range(n):
            for k, (s, flat, ones) in enumerate(sess):
                step(s, flat, ones)
                cur = s.step_end()
                if prev[k] is not None:
                    s.check_step(prev[k])
                prev[k] = cur
        for k, (s, _, _) in enumerate(sess):
            s.check_step(prev[k])
    run(3)
    t0 = time.perf_counter()
    run(20)
    dt = (time.perf_counter() - t0) / 20
    print(f"S={S}: {dt*1e3:.3f} ms/step, {npsr/dt:.0f} fits/s", flush=True)
    for s, _, _ in sess:
        s.close()
