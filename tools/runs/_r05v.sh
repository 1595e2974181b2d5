#!/bin/bash
# round 5 (v): the profile set again on another box (r05u's box ran every kernel 4 - 35 % slower)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05v bench prof pmc sq side
