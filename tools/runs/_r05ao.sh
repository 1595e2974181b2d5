#!/bin/bash
# round 5 (ao): final-tree profile set (24-row head conv tiles, ABI 14) -- rocprofv3 kernel stats, FETCH/WRITE + SQ PMC passes,
# side-encoder ablation, the video loops (configs 3 and 5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05ao bench prof pmc sq side loop
