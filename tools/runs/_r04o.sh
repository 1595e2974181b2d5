cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04o && mkdir -p $O && \
bash tools/ab_env.sh r04o_ab "DP_X=0" "DP_GEMM_DEBUG=134217728" "DP_GEMM_DEBUG=268435456" "DP_GEMM_DEBUG=536870912"
