#!/bin/bash
# round 5 (ak): current-tree profile set -- rocprofv3 kernel stats, FETCH/WRITE + SQ PMC passes,
# side-encoder ablation, the video loops (configs 3 and 5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05ak bench prof pmc sq side loop
