cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04t && mkdir -p $O && \
DP_GEMM_DEBUG=134217728 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -s --timeout 300 --timeout-method thread -k "grouped" > $O/pytest_grp2.log 2>&1 && \
bash tools/ab_env.sh r04t_ab "DP_X=0" "DP_GEMM_DEBUG=134217728"
