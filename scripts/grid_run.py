"""The bench's chi2-grid leg alone (NGC6440E, side x side (F0, F1), WLSFitter per point),
for a kernel trace of the grid's launches without the PTA leg's (rocprofv3 --kernel-trace
--stats -- python3 scripts/grid_run.py 256)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

if __name__ == "__main__":
    from pint_amd import _lib
    _lib.lib()
    import bench
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    print(json.dumps(bench.grid_leg(side, None, lambda: None, lambda v: v)))
