#!/bin/bash
# round 5 (av): proj / fc2 split producer streaming its epilogue's residual rows during the K loop
# (touch LDS-DMA; debug 1 << 28: off): parity, alone (warm / cold), in-frame A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05av
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "8ph320 or split_producer or split_residual" > gpurun_out/r05av/tests.log 2>&1 || { tail -30 gpurun_out/r05av/tests.log; exit 1; }
tail -1 gpurun_out/r05av/tests.log
timeout -k 10 200 python -u tools/hilo_bench.py > gpurun_out/r05av/hilo.txt 2>&1
grep -v amdgpu.ids gpurun_out/r05av/hilo.txt | tr '|' '\n'
bash tools/ab_env.sh r05av_ab "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=268435456"
