#!/bin/bash
# round 6 (h): the LN-consumer GEMMs (qkv, fc1) on the 8-phase 320 x 256 engine (debug 1 << 25)
# now that its K loop is faster -- fc1 alone both ways, in-frame A/B alternating
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
for R in 1 2; do
  timeout -k 10 120 python -u tools/fc1_bench.py --dbg 33554432 2>/dev/null >> $O/fc1_alone.txt
done
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/ab_p8_$R.json 2> $O/ab_p8_$R.err
  DP_GEMM_DEBUG=33554432 timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $O/ab_320_$R.json 2> $O/ab_320_$R.err
done
python3 - <<'PY' > $O/ab.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/r06h/ab_*.json")):
    d = json.load(open(f)); print(f, d.get("value"), d.get("ab_fps"), d.get("ms_per_step"), (d.get("parity") or {}).get("depth_rel_l1"))
PY
