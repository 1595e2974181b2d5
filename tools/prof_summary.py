#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (SQLite .db or kernel_stats.csv) as markdown."""
import csv
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\((anonymous namespace)?::?GemmP\)|\(.*\)$", "", name)
    return name[:110]


def rows_from(path: str):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
            yield r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4])
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                       float(r["AverageNs"]) / 1e3, float(r["Percentage"]))


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(path)
    print(f"# {title}\n\nsource: `{path}` (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | calls | total us | avg us | % |\n|---|---:|---:|---:|---:|")
    for name, calls, tot, avg, pct in rows_from(path):
        if pct < 0.01:
            continue
        print(f"| `{short(name)}` | {calls} | {tot:.1f} | {avg:.2f} | {pct:.2f} |")


if __name__ == "__main__":
    main()
