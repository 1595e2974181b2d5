#!/bin/bash
# round 6 (o): what bounds the composed head (head.ps, 512 x 128 implicit-conv engine): timing ablations
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o; mkdir -p $O
for R in 1 2; do
  timeout -k 10 200 python -u tools/head_bench.py --ablate 2>/dev/null >> $O/head_ablate.txt
done
