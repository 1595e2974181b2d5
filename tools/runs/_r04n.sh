cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04n && mkdir -p $O && \
timeout -k 10 300 python -u tools/frame_shapes.py > $O/shapes_splitk.txt 2>&1 && \
DP_GEMM_DEBUG=134217728 timeout -k 10 300 python -u tools/frame_shapes.py > $O/shapes_nosplitk.txt 2>&1 && \
bash tools/ab_env.sh r04n_ab "DP_X=0" "DP_GEMM_DEBUG=134217728"
