"""Instruction mix of the MFMA loops of a kernel in a device assembly listing.

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S pint_hip.hip -o pint.s
    python scripts/diag/isa_loops.py pint.s k_gram_vILi2ELi6ELb1E [--all]

Prints, per loop (a label with a backward branch to it) that holds an MFMA (or every loop
with --all), the instruction count by class and the scratch/vmcnt waits in it."""
import collections
import re
import sys


def body_of(lines, key):
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + key + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_") and "f64" in op:
        return "v_f64"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "v_lane"
    if op.startswith("v_"):
        return "v_other"
    if op.startswith("ds_"):
        return "ds_" + ("write" if "write" in op else "read" if "read" in op else "other")
    if op.startswith(("global_", "buffer_")):
        return "gmem"
    if op.startswith("scratch_"):
        return "SCRATCH"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return op


def main():
    path, key = sys.argv[1], sys.argv[2]
    allloops = "--all" in sys.argv
    L = body_of(open(path).read().split("\n"), key)
    labels = {}
    for i, l in enumerate(L):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    seen = set()
    for i, l in enumerate(L):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if not m or m.group(1) not in labels or labels[m.group(1)] >= i:
            continue
        a = labels[m.group(1)]
        if a in seen:
            continue
        seen.add(a)
        ins = [x.split()[0] for x in L[a:i + 1] if x.startswith("\t") and not x.strip().startswith((".", ";"))]
        c = collections.Counter(klass(op) for op in ins)
        if c["mfma"] or allloops:
            valu = sum(v for k, v in c.items() if k.startswith("v_") or k == "mfma")
            print(f"{m.group(1)} lines {a}-{i}: {len(ins)} instr, VALU {valu} (per MFMA "
                  f"{valu / max(c['mfma'], 1):.1f}) {dict(sorted(c.items(), key=lambda kv: -kv[1]))}")


if __name__ == "__main__":
    main()
