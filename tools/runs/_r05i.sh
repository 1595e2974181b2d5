#!/bin/bash
# round 5 (i): the patch encoder's folded qkv on the persistent 8-phase engine (DP_QKV_P8=1): A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05i
DP_QKV_P8=1 timeout -k 10 200 python -u -X faulthandler tools/dbg_sched.py > gpurun_out/r05i/dbg.log 2>&1
bash tools/ab_env.sh r05i "DP_QKV_P8=0" "DP_QKV_P8=1"
