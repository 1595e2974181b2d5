#!/bin/bash
# round 5 (ay): the side encoders' grouped GEMMs on 128 x 128 tiles (default) vs 256 x 128 (debug 1 << 26)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05ay "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=67108864" "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=67108864"
