#!/bin/bash
# round 5 (au): side-encoder cost by ablation on one box, 4 alternating samples each
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05au "DP_NOTHING=1" "DP_ABLATE=side" "DP_NOTHING=1" "DP_ABLATE=side"
