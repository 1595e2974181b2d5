#!/bin/bash
# round 6 (m): full-tree check on the final kernels -- GPU tests, smoke, bench
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r06m tests smoke bench
