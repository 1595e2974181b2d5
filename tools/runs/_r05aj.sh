#!/bin/bash
# round 5 (aj): current tree (convs.4 on split-K) -- GPU tests, smoke, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05aj tests smoke bench
