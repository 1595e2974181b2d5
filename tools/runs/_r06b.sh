#!/bin/bash
# round 6 (b): pruned tree, ln_rs clamp fix, same-size resize copy -- GPU tests + bench
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r06b tests bench
