#!/usr/bin/env python3
"""Summary of a tools/frame_timeline_cc.py --all listing: per (kind, shape) on the main stream in the
patch-encoder part (before the last fc2 ends), the in-frame launch times, and the idle gaps between
consecutive main-stream launches.

    python tools/timeline_summary.py gpurun_out/<tag>/timeline_all.txt
"""
import collections
import sys


def main():
    path = sys.argv[1]
    lines = [ln for ln in open(path).read().splitlines() if "amdgpu.ids" not in ln]
    t_enc = float(lines[0].split("patch encoder ends at ")[1].split()[0])
    rows = []
    for ln in lines[1:]:
        f = ln.split()
        if not f or f[0] not in ("main", "side", "dec_a", "dec_b", "dec_c"):
            continue
        rows.append((f[0], float(f[1]), float(f[2]), f[7], " ".join(f[8:])))
    main_rows = sorted(r for r in rows if r[0] == "main" and r[2] <= t_enc + 1e-6)
    d = collections.defaultdict(list)
    for r in main_rows:
        d[(r[3], r[4])].append(1000 * (r[2] - r[1]))
    print(f"patch-encoder part (main stream, in-frame): 0 .. {t_enc:.3f} ms")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"  {k[0]:12s} {k[1]:28s} n={len(v):3d} avg {sum(v) / len(v):7.1f} us  total {sum(v) / 1000:6.3f} ms")
    gaps = [b[1] - a[2] for a, b in zip(main_rows, main_rows[1:])]
    gaps.sort()
    print(f"  gaps between main-stream launches: n={len(gaps)} total {sum(gaps):.3f} ms, median "
          f"{1000 * gaps[len(gaps) // 2]:.2f} us, max {1000 * gaps[-1]:.2f} us")
    side = [r for r in rows if r[0] == "side"]
    if side:
        print(f"  side stream: {len(side)} launches, {sum(1000 * (r[2] - r[1]) for r in side) / 1000:.3f} ms of "
              f"stream time, ends at {max(r[2] for r in side):.3f} ms")


if __name__ == "__main__":
    main()
