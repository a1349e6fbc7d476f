"""The drop-in boundary from real PINT objects (pint_amd.interop), checked in the build
container against the reference itself: oracle/refgen/check_interop.py loads NGC6440E and
B1855+09 with PINT (/root/reference, offline recipe), converts them with
interop.from_pint, and compares the packed columns, the TZR TOA and every parameter with
the committed fixtures (which the reference wrote), and the CPU oracle's residuals of the
converted objects with the reference's.  Skipped where the reference is absent (GPU box)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "oracle", "refenv", "run_ref.sh")


@pytest.mark.skipif(not (os.path.isdir("/root/reference/src/pint") and os.path.exists("/opt/conda/bin/python3.9")),
                    reason="needs the reference PINT and its interpreter (build container only)")
def test_from_pint_matches_reference_fixtures():
    p = subprocess.run(["bash", RUN, "check_interop.py"], cwd=os.path.join(ROOT, "oracle", "refgen"),
                       capture_output=True, text=True, timeout=900)
    line = [l for l in p.stdout.splitlines() if l.startswith("INTEROP ")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    res = json.loads(line[0][len("INTEROP "):])
    for name, r in res.items():
        assert max(r["columns_maxrel"].values()) <= 1e-15, (name, r["columns_maxrel"])
        assert all(r["tzr_equal"].values()), (name, r["tzr_equal"])
        assert r["param_mismatch"] == {}, (name, r["param_mismatch"])
        assert r["free_params_equal"], name
        assert r["resid_max_abs_s"] < 1e-10, (name, r["resid_max_abs_s"])  # bar 1 ns
