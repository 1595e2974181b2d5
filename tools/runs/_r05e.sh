#!/bin/bash
# round 5 (e): profile of the tree after the split residual: bench line, rocprofv3 kernel stats,
# FETCH/WRITE + SQ PMC passes, side-encoder ablation
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05e bench prof pmc sq side
