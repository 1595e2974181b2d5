cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04v && mkdir -p $O && \
DP_GEMM_DEBUG=134217728 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -v -s --timeout 300 --timeout-method thread -k "layernorm or stages" > $O/pytest_ln4.log 2>&1 && \
bash tools/ab_env.sh r04v_ab "DP_X=0" "DP_GEMM_DEBUG=134217728"
