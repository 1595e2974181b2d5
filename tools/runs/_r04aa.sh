cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04aa && mkdir -p $O && \
DP_GEMM_DEBUG=134217728 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread -k "grouped" > $O/pytest_ns4.log 2>&1 && \
DP_GEMM_DEBUG=268435456 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread -k "grouped" > $O/pytest_ns5.log 2>&1 && \
bash tools/ab_env.sh r04aa_ab "DP_X=0" "DP_GEMM_DEBUG=134217728" "DP_GEMM_DEBUG=268435456"
