#!/bin/bash
# round 5 (as): final tree (HEAD_PS hints) -- GPU tests, smoke, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05as tests smoke bench
