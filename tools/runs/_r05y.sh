#!/bin/bash
# round 5 (y): the patch-conv engine on 12 x 16-pixel tiles for the 384^2 convs (DP_TILE_CV3_192x256):
# kernel tests, stamps, alone timing, in-frame A/B (debug 1 << 30: the 320 x 256 engine as before)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05y
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -m gpu \
  -k "patch_conv" > gpurun_out/r05y/pytest.log 2>&1
timeout -k 10 100 python -u tools/cv3_stamps.py --size 384 --th 12 --seconds 1 > gpurun_out/r05y/stamps12.txt 2>&1
timeout -k 10 100 python -u tools/cv3_stamps.py --size 384 --th 16 --seconds 1 > gpurun_out/r05y/stamps16.txt 2>&1
timeout -k 10 200 python -u tools/gemm_bench.py --only "rb conv 384" --tile big320x256,cv3_256x256,cv3_192x256 > gpurun_out/r05y/conv384.txt 2>&1
bash tools/ab_env.sh r05y "DP_GEMM_DEBUG=1073741824" "DP_GEMM_DEBUG=0"
