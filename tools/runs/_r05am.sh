#!/bin/bash
# round 5 (am): 24 x 16-pixel patch-conv tiles for the 128-channel head conv: parity, alone, in-frame
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05am
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "patch_conv" > gpurun_out/r05am/tests.log 2>&1 || { tail -30 gpurun_out/r05am/tests.log; exit 1; }
tail -1 gpurun_out/r05am/tests.log
for r in 1 2; do
  for d in 0 536870912; do
    echo "== DP_GEMM_DEBUG=$d" >> gpurun_out/r05am/head_alone.txt
    DP_GEMM_DEBUG=$d timeout -k 10 120 python -u tools/head_bench.py >> gpurun_out/r05am/head_alone.txt 2>&1
  done
done
grep -v amdgpu.ids gpurun_out/r05am/head_alone.txt
bash tools/ab_env.sh r05am_ab "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=536870912"
