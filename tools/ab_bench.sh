#!/bin/bash
# In-frame A/B of DP_GEMM_DEBUG switches: bench.py alternating the given flag sets, 2 rounds.
# Usage (on the gpurun box, repo root): tools/ab_bench.sh <tag> <flags-A> <flags-B> [<flags-C> ...]
set -eo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for R in 1 2; do
  for F in "$@"; do
    DP_GEMM_DEBUG=$F timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $OUT/ab_${F}_$R.json 2> $OUT/ab_${F}_$R.err
  done
done
python - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.load(open(f))
    dk = d["roofline"]["dominant_kernel"]
    print(f.split("/")[-1], d["ab_fps"], d["ms_per_step"], d["parity"]["depth_rel_l1"], dk["engine"]["tile"], dk["avg_us"])
PY
