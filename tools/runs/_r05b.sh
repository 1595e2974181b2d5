#!/bin/bash
# round 5 (b): split-residual epilogue with 3 chunks of DMA in flight vs 1 -- tests, micro-bench, in-frame A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r05b && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "layernorm_stats or ln_producer or split_residual" > $O/pytest_kern.log 2>&1 && \
timeout -k 10 200 python -u tools/hilo_bench.py > $O/hilo_bench.txt 2>&1 && \
DP_TEST_METRICS=$O/test_metrics.json timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -v \
  --timeout 300 --timeout-method thread -k "forward_frame0 or stage_parity" > $O/pytest_model.log 2>&1 && \
bash tools/ab_env.sh r05b_ab "DP_GEMM_DEBUG=0" "DP_GEMM_DEBUG=134217728"
