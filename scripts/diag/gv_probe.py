"""k_gram_v phase experiment: the bench's 68 x 10k PTA step with phases of k_gram_v switched
off (option 99 bits: 1 = no global loads in the stager loop, 2 = no MFMAs, 4 = no staging);
prints the Gram event time per step for each."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from pint_amd import simulation as sim
from pint_amd.engine import Session, build_layout, pack_table

models = [sim.pta_model(i) for i in range(68)]
items = sim.make_pta(ntoas=10000, indices=list(range(68)), models=models)
s = Session(device=0)
lays = [s.add(build_layout(m, t)) for m, t in items]
tabs0 = [pack_table(l, m) for l, (m, _) in zip(lays, items)]
s.set_instances(list(zip(lays, tabs0)))
flat0 = np.concatenate(tabs0)
print("nsplit", s.nsplit(), flush=True)
s.set_timing_mask(1 << 6)
for dbg in [0, 1, 2, 3, 4, 5, 6, 7, 0]:
    s.L.pint_set_option(s.ctx, 99, dbg)
    ts = []
    for k in range(6):
        s.set_tables(flat0)
        s.eval(want_M=Session.FIT)
        try:
            s.fit_step(1)
            s.check()
        except Exception:
            pass
        ts.append(s.timing()[6])
    print(f"dbg {dbg}: gram ms {np.median(ts[2:]):.4f}", flush=True)
s.L.pint_set_option(s.ctx, 99, 0)
s.close()

# per-workgroup timeline of k_gram_v (option bit 8)
s = Session(device=0)
lays = [s.add(build_layout(m, t)) for m, t in items]
s.set_instances(list(zip(lays, tabs0)))
for dbg in [8, 8 | 2, 8 | 7]:
    s.L.pint_set_option(s.ctx, 99, dbg)
    for k in range(3):
        s.set_tables(flat0)
        s.eval(want_M=Session.FIT)
        try:
            s.fit_step(1)
            s.check()
        except Exception:
            pass
    out = np.zeros(4096 * 5)
    import ctypes
    s.L.pint_debug_read(s.ctx, 5, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    nb = 68 * s.nsplit()
    t = out[:nb * 5].reshape(nb, 5)
    t0 = t[:, 0].min()
    st, pro, lp, end, cu = (t[:, 0] - t0) * 0.01, (t[:, 1] - t[:, 0]) * 0.01, (t[:, 2] - t[:, 1]) * 0.01, \
        (t[:, 3] - t[:, 2]) * 0.01, t[:, 4]
    print(f"dbg {dbg}: span {((t[:, 3].max() - t0) * 0.01):.1f} us; per block: prologue {np.median(pro):.2f} "
          f"loop {np.median(lp):.2f} (min {lp.min():.2f} max {lp.max():.2f}) epilogue {np.median(end):.2f} us; "
          f"start times quantiles {np.quantile(st, [0, .25, .5, .75, 1]).round(1)}; distinct cu ids {len(np.unique(cu))}",
          flush=True)
    np.save(f"gpurun_out/gvts_{dbg}.npy", t)
s.close()
