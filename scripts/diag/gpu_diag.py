"""Diagnostic parity run against all golden fixtures (prints, does not assert)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from golden_util import load, ref_value
from pint_amd import Residuals, WLSFitter, GLSFitter
from pint_amd.engine import evaluate_delay_phase

names = sys.argv[1:] or ["ngc6440e", "pta_iso", "pta_ell1", "pta_dd", "j0740", "b1855"]
for name in names:
    print("=====", name, flush=True)
    try:
        model, toas, z, meta = load(name)
        t0 = time.time()
        dp = evaluate_delay_phase(model, toas)
        d = dp["delay"] - z["delay_total"]
        print(f"delay max|d| {np.abs(d).max():.3e} s  tzr delay {dp['tzr_delay']:.12f} vs {z['tzr_delay'][0]:.12f}")
        r = Residuals(toas, model)
        dr = r.time_resids - z["res_time"]
        print(f"resid max|d| {np.abs(dr).max():.3e} s  rms {np.sqrt(np.mean(dr**2)):.3e}  chi2 {r.chi2:.10g} ref {meta['res_chi2']:.10g} rel {(r.chi2-meta['res_chi2'])/meta['res_chi2']:.3e}  track {r.track_mode}")
        M, params, units = model.designmatrix(toas)
        Mr = z["dm_M"]
        rows = z["dm_rows"] if "dm_rows" in z else np.arange(M.shape[0])
        worst = []
        for j, p in enumerate(params):
            if p not in meta["dm_params"]:
                worst.append((p, "missing-in-ref")); continue
            jr = meta["dm_params"].index(p)
            a = M[rows, j]; b = Mr[:, jr]
            sc = np.abs(b).max() or 1.0
            worst.append((p, np.abs(a - b).max() / sc))
        worst.sort(key=lambda x: -x[1] if isinstance(x[1], float) else 0)
        print("designmatrix worst rel col err:", [(p, f"{e:.2e}" if isinstance(e, float) else e) for p, e in worst[:6]])
        if "wls_chi2" in meta:
            f = WLSFitter(toas, model)
            c2 = f.fit_toas(maxiter=1)
            print(f"WLS chi2 {c2:.10g} ref {meta['wls_chi2']:.10g} rel {(c2-meta['wls_chi2'])/meta['wls_chi2']:.2e}")
            for p in meta["wls_params"]:
                v = f.model[p].value; rv = ref_value(meta, "wls_params", p); s = meta["wls_errors"][p]
                print(f"   {p}: dpar/sigma {float((np.longdouble(v) - rv)/np.longdouble(s)):.2e}  err ratio {f.model[p].uncertainty/s:.6f}")
        if "gls_chi2" in meta:
            f = GLSFitter(toas, model)
            c2 = f.fit_toas(maxiter=1)
            print(f"GLS chi2 {c2:.10g} ref {meta['gls_chi2']:.10g} rel {(c2-meta['gls_chi2'])/meta['gls_chi2']:.2e}")
            mx = 0; me = 0
            for p in meta["gls_params"]:
                v = f.model[p].value; rv = ref_value(meta, "gls_params", p); s = meta["gls_errors"][p]
                x = abs(float((np.longdouble(v) - rv)/np.longdouble(s))); mx = max(mx, x)
                me = max(me, abs(f.model[p].uncertainty/s - 1))
            print(f"   max |dpar|/sigma {mx:.2e}  max |err ratio-1| {me:.2e}")
        print(f"   ({time.time()-t0:.1f}s)")
    except Exception as e:
        import traceback; traceback.print_exc()
