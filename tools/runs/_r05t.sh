#!/bin/bash
# round 5 (t): split-residual epilogue DMA depth 1 vs 3 (debug 1 << 27) on the current tree, 3 rounds
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05t "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=134217728"
bash tools/ab_env.sh r05t2 "DP_GEMM_DEBUG=134217728" "DP_GEMM_DEBUG=0"
