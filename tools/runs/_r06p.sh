#!/bin/bash
# round 6 (p): the bench line of the final tree with the committed r06 profile set it cites
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r06p smoke bench
