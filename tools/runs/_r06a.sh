#!/bin/bash
# round 6 (a): pruned tree + pipelined attention -- GPU tests + bench; attention A/B (pipelined vs tile loop)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1
for R in 1 2; do for P in 0 1; do for S in 577 640; do
  echo "pipe=$P" >> $O/attn_ab.txt
  DP_ATTN_PIPE=$P timeout -k 10 120 python -u tools/attn_bench.py --quick --log2q --seq $S >> $O/attn_ab.txt 2>&1
done; done; done
bash tools/gpu_check.sh r06a tests bench
