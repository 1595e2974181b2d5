#!/bin/bash
# round 5 (o): is the side chain's latency on the critical path? side LayerNorms skipped vs full vs no side
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh r05o "DP_ABLATE=" "DP_ABLATE=sideln" "DP_ABLATE=side"
