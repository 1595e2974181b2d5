#!/bin/bash
# round 5 (aq): the composed depth head (HEAD_PS) on 24-row patch-conv tiles vs the 512 x 128 engine
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05aq
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "patch_conv3x3_head" > gpurun_out/r05aq/tests.log 2>&1 || { tail -30 gpurun_out/r05aq/tests.log; exit 1; }
tail -1 gpurun_out/r05aq/tests.log
for r in 1 2; do
  for t in 0 23; do
    echo "== HEAD_PS_TILE=$t" >> gpurun_out/r05aq/head_alone.txt
    HEAD_PS_TILE=$t timeout -k 10 120 python -u tools/head_bench.py >> gpurun_out/r05aq/head_alone.txt 2>&1
  done
done
grep -v amdgpu.ids gpurun_out/r05aq/head_alone.txt
