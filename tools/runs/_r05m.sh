#!/bin/bash
# round 5 (m): producer-merged LN row statistics (ABI 13, DP_LN_RS): kernel + model tests, A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05m
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 300 \
  --timeout-method thread -m gpu -k "merged_row_stats or split_residual or ln_consumer or layernorm_stats or mixed" \
  > gpurun_out/r05m/pytest.log 2>&1
bash tools/ab_env.sh r05m "DP_LN_RS=0" "DP_LN_RS=1"
