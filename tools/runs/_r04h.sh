cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04h && mkdir -p $O && \
DP_GEMM_DEBUG=67108864 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -s --timeout 300 --timeout-method thread -k "grouped" > $O/pytest_grp128.log 2>&1 && \
bash tools/ab_env.sh r04h_ab "DP_X=0" "DP_GEMM_DEBUG=67108864" "DP_ABLATE=side"
