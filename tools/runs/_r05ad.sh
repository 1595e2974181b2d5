#!/bin/bash
# round 5 (ad): kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) for the graph's launches
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05ad2 "DP_NOTHING=1" "HIP_FORCE_DEV_KERNARG=1"
