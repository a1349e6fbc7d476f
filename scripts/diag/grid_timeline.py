"""Device timeline of one chi2 grid from a rocprofv3 kernel (+ memory copy) trace of
scripts/grid_run.py: dispatches and copies grouped into grids by idle gaps > GAP us; prints
the kernels and copies of grid IDX (0 = first) with start offset, duration and queue.
    python3 scripts/diag/grid_timeline.py TRACE_DIR [IDX]"""
import csv
import glob
import sys

GAP = 150.0
d = sys.argv[1]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:34],
                   r.get("Queue_Id", "?")))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")[:20] +
                   f" {int(r.get('Size', 0)) / 1024:.0f}KB", "c"))
ev.sort()
groups, cur, last = [], [], None
for e in ev:
    if last is not None and (e[0] - last) / 1e3 > GAP:
        groups.append(cur)
        cur = []
    cur.append(e)
    last = max(last or 0, e[1])
groups.append(cur)
def busy_of(g):
    b, end = 0.0, g[0][0]
    for s, e, _, _ in g:
        b += max(0, e - max(s, end))
        end = max(end, e)
    return b / 1e3


if idx < 0:
    for i, g in enumerate(groups):
        if len(g) > 6:
            print(f"group {i:3d}: {len(g):3d} events span {(g[-1][1] - g[0][0]) / 1e3:7.1f} us busy {busy_of(g):7.1f} us  "
                  f"first {g[0][2]} ... {g[-1][2]}")
    sys.exit(0)
g = groups[idx]
t0 = g[0][0]
busy = 0.0
end = t0
for s, e, n, q in g:
    print(f"  +{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  q{q:>3s}  {n}")
    busy += max(0, e - max(s, end))
    end = max(end, e)
print(f"span {(g[-1][1] - t0) / 1e3:.1f} us, device busy (union) {busy / 1e3:.1f} us")
