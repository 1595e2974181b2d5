#!/bin/bash
# round 5 (ac): final-tree profile set after the 12-row patch-conv tiles: bench, rocprofv3 kernel stats,
# FETCH/WRITE + SQ PMC passes, side-encoder ablation, the video loops (configs 3 and 5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05ac bench prof pmc sq side loop
