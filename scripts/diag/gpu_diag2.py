import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from golden_util import load
from pint_amd.engine import Session, build_layout, pack_table
from pint_amd import _lib as L
from pint_amd.noise import fourier_basis, red_noise_freqs_weights

for name in sys.argv[1:]:
    model, toas, z, meta = load(name)
    s = Session()
    lay = s.add(build_layout(model, toas))
    s.set_instances([(lay, pack_table(lay))])
    s.eval(True)
    hi, lo, ft, dl = [x[0] for x in s.read_eval()]
    ph = np.longdouble(hi) + np.longdouble(lo)
    rel = ph[:-1] - ph[-1]
    ref = np.longdouble(z["phase_int"]) + np.longdouble(z["phase_frac_hi"]) + np.longdouble(z["phase_frac_lo"])
    d = (rel - ref).astype(float)
    print(name, "abs phase diff cycles: max", np.abs(d).max(), "rms", np.sqrt(np.mean(d**2)), "mean", d.mean())
    ref0 = np.longdouble(z["phase_noabs_int"]) + np.longdouble(z["phase_noabs_frac"])
    d0 = (ph[:-1] - ref0).astype(float)
    print("   noabs phase diff: max", np.abs(d0).max(), "mean", d0.mean(), " tzr phase", ph[-1])
    print("   first rows diff", d[:5], d0[:5])
    M = s.read_designmatrix()[0]
    if lay.nred:
        F = fourier_basis(model, toas)
        print("   F cols max abs diff", np.abs(M[:, len(lay.columns):] - F).max())
    s.fit_step(1 if lay.nred else 0)
    G = np.empty(s.L.pint_debug_read(s.ctx, 0, None) if False else 0)
    nsplit = 0
    Gp = np.empty(10**7)
    nsplit = s.L.pint_debug_read(s.ctx, 0, L.ptr(Gp))
    Kp = ((lay.K + 1 + 15) // 16) * 16
    G = Gp[: nsplit * Kp * Kp].reshape(nsplit, Kp, Kp).sum(0)
    T = np.hstack([M, s.read_resids()[0][0][:, None]])
    w = 1.0 / (lay.sigma_us * 1e-6) ** 2
    Gn = T.T @ (w[:, None] * T)
    K1 = lay.K + 1
    Gu = np.triu(G[:K1, :K1])
    Gnu = np.triu(Gn)
    print("   nsplit", nsplit, "Gram rel err (upper):", np.abs(Gu - Gnu).max() / np.abs(np.diag(Gn)).max(),
          "diag rel", np.max(np.abs(np.diag(Gu) - np.diag(Gn)) / np.abs(np.diag(Gn))))
    cs = np.empty(10**6)
    s.L.pint_debug_read(s.ctx, 1, L.ptr(cs))
    csq = cs[: (lay.K + 1) * nsplit].reshape(lay.K + 1, nsplit).sum(1)[: lay.K]
    print("   colsq rel err", np.max(np.abs(csq - (M ** 2).sum(0)) / (M ** 2).sum(0)))
    s.close()
