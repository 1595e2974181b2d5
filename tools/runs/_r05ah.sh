#!/bin/bash
# round 5 (ah): the decoder's 1024 -> 256 projections on the split-K engine (convs.4 / convs.3 + .4)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05ah4 "DP_SPLITK_DEC=4" "DP_SPLITK_DEC=4r" "DP_SPLITK_DEC=4" "DP_SPLITK_DEC=4r"
