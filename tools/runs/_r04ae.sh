cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ae && mkdir -p $O && \
bash tools/ab_env.sh r04ae_ab "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8"
