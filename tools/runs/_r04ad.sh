cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ad && mkdir -p $O && \
bash tools/ab_env.sh r04ad_ab "DP_PREFETCH=1" "DP_PREFETCH=0"
