#!/bin/bash
# round 5 (c): fc1 on the half-tile persistent engine (epilogue under the next K loop) -- bit-identity
# tests, fc1 micro-bench, parity, in-frame A/B vs the 8-phase persistent engine (debug 1 << 28)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r05c && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "p8h_half_tile or ln_consumer" > $O/pytest_kern.log 2>&1 && \
timeout -k 10 200 python -u tools/fc1_bench.py > $O/fc1_bench.txt 2>&1 && \
DP_TEST_METRICS=$O/test_metrics.json timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -v \
  --timeout 300 --timeout-method thread -k "forward_frame0 or stage_parity" > $O/pytest_model.log 2>&1 && \
bash tools/ab_env.sh r05c_ab "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=268435456"
