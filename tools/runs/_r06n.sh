#!/bin/bash
# round 6 (n): the final tree's profile set -- rocprofv3 kernel-trace stats of the bench, FETCH / WRITE
# and two SQ PMC passes over an eager forward, serial frames (budget + alone times), side ablation,
# the video loop
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r06n prof pmc sq serial side loop
