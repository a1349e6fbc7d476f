import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
from pint_amd.engine import Session, build_layout, pack_table
from pint_amd import simulation as sim
from pint_amd.timing_model import get_model
NPSR = int(sys.argv[1]) if len(sys.argv) > 1 else 68
items = sim.make_pta(ntoas=10000, indices=list(range(NPSR)))
s = Session(0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances([(l, pack_table(l, m)) for l, (m, _) in zip(lays, items)])
APPLY = len(sys.argv) > 2 and sys.argv[2] == "apply"  # the bench's step: lazy, fused apply
if APPLY:
    s.save_tables()
    s.set_lazy(True)
for it in range(3):
    if APPLY:
        s.restore_tables(); s.eval(want_M=Session.FIT); s.fit_step_apply(1, 1.0)
    else:
        s.eval(want_M=Session.FIT); s.fit_step(1)
    out = np.zeros(32); s.L.pint_debug_read(s.ctx, 4, s.L and __import__('pint_amd._lib', fromlist=['ptr']).ptr(out))
    print("phases us:", np.round(np.diff(out[:9]), 2), "total", round(out[8], 2))
    print("  diag factor %.2f us" % (out[10]-out[9]))
    print("  chol: diag0 %.2f barrier %.2f panel0 %.2f trail0 %.2f | rest-of-chol %.2f | inv step1 %.2f rest %.2f" % tuple(np.diff(np.concatenate([[out[2]], out[10:17]]))))
    print("  refine: residual %.2f b'' %.2f y %.2f update %.2f | steps %.2f" % tuple(np.diff(np.concatenate([[out[17]], out[18:22], [out[5]]]))))
    if APPLY:
        print("  S -= UU^T: MFMA wave 0 %.2f wave 14 %.2f | b' (wave 0) %.2f | phase %.2f" % (out[27] - out[1], out[29] - out[1], out[28] - out[27], out[2] - out[1]))
        print("  x phase: x_d %.2f z %.2f max+refine %.2f steps %.2f" % (out[25] - out[4], out[26] - out[25], out[21] - out[26], out[5] - out[21]))
        print("  tail: steps->setup start %.2f setup %.2f | export end (wave 1) %.2f after the steps" % (out[22] - out[5], out[23] - out[22], out[24] - out[5]))
    if APPLY:
        s.read_step(); s.check()
