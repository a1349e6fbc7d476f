import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
from pint_amd.engine import Session, build_layout, pack_table
from pint_amd import simulation as sim
from pint_amd.timing_model import get_model
specs=[]
for i in range(68):
    kind = "ELL1" if i % 6 in (1, 4) else ("DD" if i % 6 == 2 else "")
    m = get_model(sim.pta_par(i, kind))
    specs.append(dict(model=m, start=53000, end=56652, ntoas=10000, freq=[800, 1200, 1600, 2000], obs="geocenter", error_us=0.5, add_noise=True, add_correlated_noise=True, seed=i))
toas = sim.make_fake_toas_batch(specs)
s = Session(0)
lays = [s.add(build_layout(sp["model"], t)) for sp, t in zip(specs, toas)]
s.set_instances([(l, pack_table(l, sp["model"])) for l, sp in zip(lays, specs)])
for it in range(2):
    s.eval(want_M=Session.FIT); s.fit_step(1)
    out = np.zeros(32); s.L.pint_debug_read(s.ctx, 4, s.L and __import__('pint_amd._lib', fromlist=['ptr']).ptr(out))
    print("phases us:", np.round(np.diff(out[:9]), 2), "total", round(out[8], 2))
    print("  diag factor %.2f us" % (out[10]-out[9]))
    print("  chol: diag0 %.2f barrier %.2f panel0 %.2f trail0 %.2f | rest-of-chol %.2f | inv step1 %.2f rest %.2f" % tuple(np.diff(np.concatenate([[out[2]], out[10:17]]))))
    print("  refine: residual %.2f b'' %.2f y %.2f update %.2f | steps %.2f" % tuple(np.diff(np.concatenate([[out[17]], out[18:22], [out[5]]]))))
