cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r01l && \
bash tools/frame_ablation.sh > gpurun_out/r01l/ablation.log 2>&1
