"""profiles/pmc_grid_rNN.json from rocprofv3 --pmc passes of scripts/grid_run.py (the bench's
NGC6440E 256 x 256 (F0, F1) WLS grid): per-launch HBM bytes (FETCH_SIZE x 2 on gfx950 +
WRITE_SIZE, MI355X_MICROARCH.md) and VALU issue utilisation of each grid kernel.

  valu_busy_frac  SQ_INSTS_VALU x 4 cycles (a 64-lane VALU instruction on a 16-lane SIMD) /
                  (1024 SIMDs x kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs

Kernel names follow bench.grid_roofline: k_eval_M / k_eval (k_eval<1|0, model> and the
merged k_eval_mix; for a spin-only grid k_eval_M is k_eval_head + k_eval_spin), k_resid (k_resid1 + k_resid2: one residual pass), k_gram (k_gram_s or
k_gram), k_solve (k_solve_blk).  A launch's value is the mean over its dispatches.

usage: pmc_grid_summary.py OUT FETCH_DIR WRITE_DIR VALU_DIR
"""
import collections
import csv
import json
import re
import sys

SIMDS, XCDS = 1024, 8


def key(name):
    n = name.split("(")[0].replace("void ", "").strip()
    if n.startswith("k_eval_spin") or n.startswith("k_eval_head"):
        return "k_eval_M"  # a spin-only grid's evaluation with M: the shared head, then each point's spin part
    m = re.match(r"k_eval(_mix)?(_w)?<(\d)", n)
    if m:
        return "k_eval_M" if m.group(3) == "1" else "k_eval"
    if n.startswith("k_resid1") or n.startswith("k_resid2"):
        return "k_resid"
    if n.startswith("k_gram"):
        return "k_gram"
    if n.startswith("k_solve"):
        return "k_solve"
    return re.sub(r"<.*", "", n)


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        full = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if full.startswith("__amd"):
            continue
        per[key(full)][full][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # a spin-only grid's evaluation with M is k_eval_head + k_eval_spin; a full k_eval<1, ..>
    # dispatch beside them is the one-pulsar fit before the grid, not a grid launch
    em = per.get("k_eval_M", {})
    if any(f.startswith("k_eval_spin") for f in em):
        for f in [f for f in em if not (f.startswith("k_eval_spin") or f.startswith("k_eval_head"))]:
            del em[f]
    # a launch: the sum over the group's kernels of their per-dispatch means
    out = collections.defaultdict(dict)
    for k, byname in per.items():
        cnt = collections.defaultdict(float)
        for full, ctrs in byname.items():
            for c, v in ctrs.items():
                cnt[c] += sum(v) / len(v)
        out[k] = dict(cnt)
    return out


def main(out, fdir, wdir, vdir):
    f, w, v = load(fdir), load(wdir), load(vdir)
    res = {}
    for k in sorted(set(f) | set(w) | set(v)):
        e = {}
        if "FETCH_SIZE" in f.get(k, {}) and "WRITE_SIZE" in w.get(k, {}):
            e["fetch_bytes"] = f[k]["FETCH_SIZE"] * 1024.0 * 2.0
            e["write_bytes"] = w[k]["WRITE_SIZE"] * 1024.0
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        vv = v.get(k, {})
        if "SQ_INSTS_VALU" in vv and vv.get("GRBM_GUI_ACTIVE"):
            cyc = vv["GRBM_GUI_ACTIVE"] / XCDS
            e["valu_insts"] = vv["SQ_INSTS_VALU"]
            e["valu_busy_frac"] = round(vv["SQ_INSTS_VALU"] * 4.0 / (SIMDS * cyc), 4)
            e["kernel_cycles"] = cyc
            if "SQ_WAVES" in vv:
                e["waves"] = vv["SQ_WAVES"]
        res[k] = e
    json.dump({"workload": "ngc6440e 256x256 (F0,F1) WLS grid (scripts/grid_run.py)", "workload_key": "ngc256",
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
