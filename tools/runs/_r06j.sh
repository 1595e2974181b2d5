#!/bin/bash
# round 6 (j): 8-row tile bands (debug 1 << 18: every engine's tile_coords) -- fc1 alone and in-frame A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06j; mkdir -p $O
for R in 1 2; do
  timeout -k 10 120 python -u tools/fc1_bench.py --dbg 262144 2>/dev/null >> $O/fc1_alone.txt
done
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/ab_b4_$R.json 2> $O/ab_b4_$R.err
  DP_GEMM_DEBUG=262144 timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $O/ab_b8_$R.json 2> $O/ab_b8_$R.err
done
python3 - <<'PY' > $O/ab.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/r06j/ab_*.json")):
    d = json.load(open(f)); print(f, d.get("value"), d.get("ab_fps"), d.get("ms_per_step"), (d.get("parity") or {}).get("depth_rel_l1"))
PY
