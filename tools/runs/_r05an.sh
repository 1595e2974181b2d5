#!/bin/bash
# round 5 (an): current tree (24-row head conv tiles, ABI 14) -- GPU tests, smoke, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05an tests smoke bench
