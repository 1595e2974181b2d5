#!/bin/bash
# round 5 (ar): the composed depth head (HEAD_PS) on the 256 x 128 engine (9 whole rounds) vs 512 x 128 (4.5)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05ar
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "patch_conv3x3_head or head_compose" > gpurun_out/r05ar/tests.log 2>&1 || { tail -30 gpurun_out/r05ar/tests.log; exit 1; }
tail -1 gpurun_out/r05ar/tests.log
for r in 1 2; do
  for t in 0 5; do
    echo "== HEAD_PS_TILE=$t" >> gpurun_out/r05ar/head_alone.txt
    HEAD_PS_TILE=$t timeout -k 10 120 python -u tools/head_bench.py >> gpurun_out/r05ar/head_alone.txt 2>&1
  done
done
grep -v amdgpu.ids gpurun_out/r05ar/head_alone.txt
