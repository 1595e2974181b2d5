#!/usr/bin/env python3
"""Per-forward kernel breakdown from a rocprofv3 kernel_trace.csv (eager bench run).

Splits the trace into forwards at each dp patchify launch, takes the median
forward, and groups its dispatches by (kernel, grid) with total/avg time.
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "")
    return n[:70]


def main(path, title=""):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fwds, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "patchify_kernel" in name:
            cur = []
            fwds.append(cur)
        if cur is not None:
            cur.append(r)
    # drop trailing dispatches after the last forward's head (keep only dp kernels)
    spans = []
    for f in fwds:
        t0 = int(f[0]["Start_Timestamp"])
        dp = [r for r in f if "at::" not in r["Kernel_Name"] and "rocclr" not in r["Kernel_Name"]]
        t1 = max(int(r["End_Timestamp"]) for r in dp)
        spans.append((t1 - t0) / 1e3)
    med = statistics.median(spans)
    idx = min(range(len(spans)), key=lambda i: abs(spans[i] - med))
    f = fwds[idx]
    groups = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in f:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        wg = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) * \
            (int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_Y"]))) * \
            (int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_Z"])))
        key = (short(r["Kernel_Name"]), wg)
        groups[key][0] += 1
        groups[key][1] += d
        busy += d
    print(f"# {title}\n\nforwards in trace: {len(fwds)}; forward span (first dp launch -> last dp end): "
          f"median {med:.0f} us; sum of kernel durations in that forward {busy:.0f} us (side stream overlaps)\n")
    print("| kernel | workgroups | calls | total us | avg us | % of sum |\n|---|---:|---:|---:|---:|---:|")
    for (name, wg), (n, t) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        if t / busy < 0.002:
            continue
        print(f"| `{name}` | {wg} | {n} | {t:.0f} | {t / n:.1f} | {100 * t / busy:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
