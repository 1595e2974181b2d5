#!/bin/bash
# In-frame A/B of environment settings (bench.py AB_KNOBS such as DP_LN_FOLD=0), alternating,
# 2 rounds, bench.py lines into gpurun_out/<tag>/ (run on the gpurun box from the repo root).
# Usage: tools/ab_env.sh <tag> "VAR=a" "VAR=b" ...
set -eo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for R in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    env $E timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $OUT/ab_${i}_$R.json 2> $OUT/ab_${i}_$R.err
  done
done
python tools/ab_summary.py "$OUT" "$@" | tee $OUT/ab.txt
