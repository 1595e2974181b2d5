#!/bin/bash
# round 5 (z): the 192^2 convs on 12-row patch-conv tiles too (debug 1 << 28): alone + in-frame A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05z
timeout -k 10 200 python -u tools/gemm_bench.py --only "rb conv 192" --tile auto,cv3_192x256 > gpurun_out/r05z/conv192.txt 2>&1
bash tools/ab_env.sh r05z "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=268435456"
