#!/bin/bash
# round 5 (aw): final tree (touch streaming behind a debug bit) -- GPU tests, smoke, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05aw tests smoke bench
