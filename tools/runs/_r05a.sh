#!/bin/bash
# round 5 (a): split-residual producer (hi + lo) -- kernel tests, micro-bench, model parity, in-frame A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r05a && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "layernorm_stats or ln_producer or split_residual or ln_consumer" > $O/pytest_kern.log 2>&1 && \
timeout -k 10 200 python -u tools/hilo_bench.py > $O/hilo_bench.txt 2>&1 && \
DP_TEST_METRICS=$O/test_metrics.json timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py -x -v \
  --timeout 300 --timeout-method thread -k "forward_frame0 or stage_parity or stressed or frame_loop_drops or concurrent_schedule" \
  > $O/pytest_model.log 2>&1 && \
bash tools/ab_env.sh r05a_ab "DP_LN_SPLIT=1" "DP_LN_SPLIT=0" && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
