#!/bin/bash
# round 5 (k): side-encoder grouped GEMMs as two 4-wave 128x128 workgroups per CU (debug 1 << 28): A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05k "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=268435456"
