#!/usr/bin/env python3
"""Per-launch durations from a rocprofv3 kernel trace, in dispatch order, for one frame: the
patch encoder's block pattern (qkv, attention, proj, fc1, fc2, ...) by kernel name + grid.

    python tools/trace_seq.py <kernel_trace.csv> [--frame -1]
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*\)$", "", n)
    return n[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # frames: split at the patchify kernel
    starts = [i for i, r in enumerate(rows) if "patchify_kernel" in r["Kernel_Name"]]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    lo = starts[k]
    hi = starts[k + 1] if k + 1 < len(starts) and k + 1 != 0 else len(rows)
    fr = rows[lo:hi]
    t0, t1 = int(fr[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in fr)
    print(f"frame {k}: {len(fr)} dispatches, span {(t1 - t0) / 1e3:.1f} us")
    agg = defaultdict(list)
    for r in fr:
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"sum of kernel durations {tot:.1f} us")
    for (name, wg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) < 0.002 * tot:
            continue
        v2 = sorted(v)
        print(f"{sum(v):9.1f} us {len(v):4d} x  avg {sum(v) / len(v):7.1f}  med {v2[len(v2) // 2]:7.1f}  "
              f"wg {wg:5d}  {name}")


if __name__ == "__main__":
    main()
