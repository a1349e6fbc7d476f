"""Per-kernel, per-launch-shape summary of a rocprofv3 --kernel-trace CSV (profiles/)."""
import collections
import csv
import json
import sys


def main(trace_csv, out):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if name.startswith("__amd"):
            continue
        shape = f'grid={r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]} wg={r["Workgroup_Size_X"]}'
        d[(name, shape)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (name, shape), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        rows.append({"kernel": name, "shape": shape, "calls": len(v), "avg_us": round(sum(v) / len(v), 2),
                     "min_us": round(min(v), 2), "max_us": round(max(v), 2), "total_us": round(sum(v), 1)})
    json.dump(rows, open(out, "w"), indent=1)
    for r in rows:
        print(f'{r["kernel"]:16s} {r["shape"]:34s} calls={r["calls"]:4d} avg={r["avg_us"]:9.2f} us')


if __name__ == "__main__":
    main(*sys.argv[1:3])
