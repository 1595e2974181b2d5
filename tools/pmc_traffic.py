#!/usr/bin/env python3
"""Per-kernel HBM traffic of one eager forward from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [--json out.json]

Passes come from `tools/gpu_check.sh ... pmc` (tools/frame_once.py, eager forwards, one
dispatch per launch).  The last forward (split at each patchify launch) is used.
gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) counts half of
the bytes of a 16-B/lane streaming read -> doubled; WRITE_SIZE (KB) is exact for
16-B/lane stores.  Rows are grouped by (kernel, grid) = one shape of one kernel.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*$", "", n).replace("void ", "")
    return n[:70]


def last_forward(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    starts = [i for i, r in enumerate(rows) if "patchify_kernel" in r["Kernel_Name"]]
    return rows[starts[-1]:] if starts else rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--json")
    args = ap.parse_args()
    f = last_forward(args.fetch, "FETCH_SIZE")
    w = last_forward(args.write, "WRITE_SIZE")
    assert len(f) == len(w), (len(f), len(w))
    g = defaultdict(lambda: {"calls": 0, "read_B": 0.0, "write_B": 0.0})
    for a, b in zip(f, w):
        assert a["Kernel_Name"] == b["Kernel_Name"]
        wg = int(a["Grid_Size"]) // max(1, int(a["Workgroup_Size"]))
        k = (short(a["Kernel_Name"]), wg)
        g[k]["calls"] += 1
        g[k]["read_B"] += 2.0 * float(a["Counter_Value"]) * 1024.0
        g[k]["write_B"] += float(b["Counter_Value"]) * 1024.0
    tot = sum(v["read_B"] + v["write_B"] for v in g.values())
    print(f"one eager forward: {len(f)} dispatches, HBM traffic {tot / 1e9:.2f} GB "
          f"(2 x FETCH_SIZE + WRITE_SIZE)\n")
    print("| kernel | workgroups | calls | read MB/launch | write MB/launch | total GB |")
    print("|---|---:|---:|---:|---:|---:|")
    out = []
    for (name, wg), v in sorted(g.items(), key=lambda kv: -(kv[1]["read_B"] + kv[1]["write_B"])):
        n = v["calls"]
        print(f"| `{name}` | {wg} | {n} | {v['read_B'] / n / 1e6:.1f} | {v['write_B'] / n / 1e6:.1f} | "
              f"{(v['read_B'] + v['write_B']) / 1e9:.3f} |")
        out.append({"kernel": name, "workgroups": wg, "calls": n, "read_bytes_per_launch": v["read_B"] / n,
                    "write_bytes_per_launch": v["write_B"] / n})
    if args.json:
        json.dump({"forward_bytes": tot, "kernels": out}, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
