"""Host-side duration of each call of the bench step (pipelined), to find calls that block."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pint_amd.engine import Session, build_layout, pack_table
from pint_amd import simulation as sim
from pint_amd.timing_model import get_model
npsr = int(sys.argv[1]) if len(sys.argv) > 1 else 68
specs = []
for i in range(npsr):
    kind = "ELL1" if i % 6 in (1, 4) else ("DD" if i % 6 == 2 else "")
    m = get_model(sim.pta_par(i, kind))
    specs.append(dict(model=m, start=53000, end=56652, ntoas=10000, freq=[800, 1200, 1600, 2000],
                      obs="geocenter", error_us=0.5, add_noise=True, add_correlated_noise=True, seed=i))
toas = sim.make_fake_toas_batch(specs)
s = Session()
lays = [s.add(build_layout(sp["model"], t)) for sp, t in zip(specs, toas)]
tabs = [pack_table(l, sp["model"]) for l, sp in zip(lays, specs)]
s.set_instances(list(zip(lays, tabs)))
s.save_tables()
s.set_lazy(True)
s.set_timing_mask(1 << 6)
names = ["restore", "eval_M", "fit_step", "read_step", "noise", "apply", "eval", "chi2_gls", "step_end", "check_step"]
acc = {n: [] for n in names}
prev = None
for it in range(30):
    T = [time.perf_counter()]
    s.restore_tables(); T.append(time.perf_counter())
    s.eval(want_M=Session.FIT); T.append(time.perf_counter())
    s.fit_step(1); T.append(time.perf_counter())
    s.read_step(); T.append(time.perf_counter())
    s.noise_resids(); T.append(time.perf_counter())
    s.apply_step_uniform(1.0); T.append(time.perf_counter())
    s.eval(want_M=False); T.append(time.perf_counter())
    s.chi2_gls(); T.append(time.perf_counter())
    cur = s.step_end(); T.append(time.perf_counter())
    if prev is not None:
        s.check_step(prev)
    T.append(time.perf_counter())
    prev = cur
    if it >= 5:
        for n, a, b in zip(names, T[:-1], T[1:]):
            acc[n].append((b - a) * 1e6)
s.check_step(prev)
tot = 0.0
for n in names:
    tot += np.median(acc[n])
    print(f"{n:12s} median {np.median(acc[n]):8.1f} us  max {np.max(acc[n]):8.1f}")
print(f"sum of medians {tot:.1f} us")
