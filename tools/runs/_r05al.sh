#!/bin/bash
# round 5 (al): side-encoder cost by ablation with and without convs.4 on split-K, one box
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05al "DP_SPLITK_DEC=0" "DP_SPLITK_DEC=0 DP_ABLATE=side" "DP_SPLITK_DEC=4" "DP_SPLITK_DEC=4 DP_ABLATE=side"
