"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py into
profiles/pmc_rNN.json: HBM bytes per launch for each kernel group.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half of the bytes
of wide coalesced streaming reads -> doubled here; WRITE_SIZE is taken as is.  Both are in
KiB.  A "launch" is one step's dispatches of a kernel: the per-dispatch means of its template
instantiations are summed (k_gram_v is launched once per layout group of a fit step)."""
import collections
import csv
import json
import re
import sys


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        m = re.match(r"void k_eval<(\d), (\d)>", name)
        mm = re.match(r"void k_eval_mix<(\d)>", name)
        if m:
            key = "k_eval_M" if m.group(1) == "1" else "k_eval"
            key += f"<{m.group(2)}>"
        elif mm:
            key = "k_eval_M" if mm.group(1) == "1" else "k_eval"
        else:
            key = re.sub(r"<.*", "", name.split("(")[0].replace("void ", "").strip())
        per[key + "|" + name.split("(")[0]].append(float(r["Counter_Value"]) * 1024.0)
    # one step's value of a kernel = sum over its template instantiations of the mean per
    # dispatch (a fit step launches k_gram_v once per layout group)
    out = collections.defaultdict(list)
    for k, v in per.items():
        out[k.split("|")[0]].append(sum(v) / len(v))
    return {k: [sum(v)] for k, v in out.items()}


def main(fetch_csv, write_csv, out, workload):
    f = load(fetch_csv, "FETCH_SIZE")
    w = load(write_csv, "WRITE_SIZE")
    kern = {}
    for key in sorted(set(f) | set(w)):
        if key.startswith("__amd"):
            continue
        rd = 2.0 * sum(f.get(key, [0])) / max(1, len(f.get(key, [])))
        wr = sum(w.get(key, [0])) / max(1, len(w.get(key, [])))
        kern[key] = {"fetch_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr, "launches": len(f.get(key, []))}
    for grp in ("k_eval", "k_eval_M"):
        parts = [k for k in kern if k.startswith(grp + "<")]
        if parts:
            kern[grp] = {x: sum(kern[k][x] for k in parts) for x in ("fetch_bytes", "write_bytes", "hbm_bytes")}
    json.dump({"workload": workload, "workload_key": workload.split(" ")[0], "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1, KiB->bytes",
               "kernels": kern}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:5])
