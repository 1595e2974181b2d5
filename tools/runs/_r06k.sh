#!/bin/bash
# round 6 (k): 8-row tile bands on the persistent engine only -- for the 16-column-tile launches
# (fc1, default now), none (debug 1 << 17 = HEAD), or every launch (1 << 21: qkv too); in-frame A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "persistent or ln_consumer" --timeout 120 --timeout-method thread > $O/pytest_p8.log 2>&1
for R in 1 2; do
  DP_GEMM_DEBUG=131072 timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $O/ab_b4_$R.json 2> $O/ab_b4_$R.err
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/ab_fc1b8_$R.json 2> $O/ab_fc1b8_$R.err
  DP_GEMM_DEBUG=2097152 timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $O/ab_allb8_$R.json 2> $O/ab_allb8_$R.err
done
python3 - <<'PY' > $O/ab.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/r06k/ab_*.json")):
    d = json.load(open(f)); print(f, d.get("value"), d.get("ab_fps"), d.get("ms_per_step"), (d.get("parity") or {}).get("depth_rel_l1"))
PY
