#!/bin/bash
# round 5 (ax): split-K placements on the final tree (convs.4 default; + convs.3; + fuse_lowres)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05ax "DP_SPLITK_DEC=4" "DP_SPLITK_DEC=34" "DP_SPLITK_DEC=4f" "DP_SPLITK_DEC=0"
