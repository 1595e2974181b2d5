#!/bin/bash
# round 5 (d): split residual with an 8-bit low part -- kernel tests, micro-bench, parity, in-frame A/B vs the fp32 stream
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r05d && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "layernorm_stats or ln_producer or split_residual" > $O/pytest_kern.log 2>&1 && \
timeout -k 10 200 python -u tools/hilo_bench.py > $O/hilo_bench.txt 2>&1 && \
DP_TEST_METRICS=$O/test_metrics.json timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py -x -v \
  --timeout 300 --timeout-method thread -k "forward_frame0 or stage_parity or stressed or config5_4k or concurrent_schedule" > $O/pytest_model.log 2>&1 && \
bash tools/ab_env.sh r05d_ab "DP_LN_SPLIT=1" "DP_LN_SPLIT=0"
