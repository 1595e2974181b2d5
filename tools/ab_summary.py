#!/usr/bin/env python3
"""Summary of an ab_env.sh run: one line per bench.py JSON (variant, file, fps, ms/step, depth
rel-L1, dominant kernel and its in-frame average).  Usage: ab_summary.py <dir> "VAR=a" "VAR=b" ..."""
import glob
import json
import sys

out, envs = sys.argv[1], sys.argv[2:]
for i, e in enumerate(envs, 1):
    for f in sorted(glob.glob(f"{out}/ab_{i}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        dk = d["roofline"]["dominant_kernel"]
        v = d["value"] if d.get("value") is not None else d.get("ab_fps")
        print(e, f.split("/")[-1], v, d["ms_per_step"], d["parity"]["depth_rel_l1"], dk["kind"], dk["avg_us"])
