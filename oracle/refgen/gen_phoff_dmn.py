"""The phoff_dmn fixture (gen_phoff.py: PHOFF frozen, PLRedNoise + PLDMNoise; reference run,
container only), generated with gen_fit_spread's imports in place so that its rebuild for the
chi2 spread (fit_spread.json) draws the same TOAs.  The simulated correlated noise of a
model with PLRedNoise and PLDMNoise depends on Python's string-hash seed (the order of the
noise bases): run both with the same PYTHONHASHSEED.
Usage: PYTHONHASHSEED=0 run_ref.sh gen_phoff_dmn.py; PYTHONHASHSEED=0 run_ref.sh gen_fit_spread.py phoff_dmn"""
import gen_phoff

_capture = gen_phoff.capture
import gen_fit_spread  # noqa: E402,F401  (replaces gen_phoff.capture with its own grab)
from refcommon import register_clockless_sites  # noqa: E402

gen_phoff.capture = _capture

if __name__ == "__main__":
    register_clockless_sites()
    gen_phoff.gen("phoff_dmn", 9, False, "gls", frozen=True, dmn=True)
