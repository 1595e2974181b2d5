#!/bin/bash
# the >2^31-element GEMM test and the GEMM kernel tests after the planner's 32-bit-offset guard
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04al && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "gemm" > $O/pytest_gemm.log 2>&1
