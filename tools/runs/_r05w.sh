#!/bin/bash
# round 5 (w): the 384^2 decoder convs (461 tiles of 320 x 256) on the persistent big engine (debug 1 << 29)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05w
timeout -k 10 200 python -u tools/gemm_bench.py --only "rb conv 384" --tile big320x256,pbig320x256 > gpurun_out/r05w/conv384.txt 2>&1
bash tools/ab_env.sh r05w "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=536870912"
