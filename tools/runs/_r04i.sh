cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04i && mkdir -p $O && \
DP_GEMM_DEBUG=134217728 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -s --timeout 300 --timeout-method thread -k "grouped" > $O/pytest_grp64.log 2>&1 && \
bash tools/ab_env.sh r04i_ab "DP_GEMM_DEBUG=67108864" "DP_GEMM_DEBUG=134217728" "DP_GEMM_DEBUG=268435456"
