cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ag && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread -k "ln_producer or ln_consumer" > $O/pytest_ln.log 2>&1 && \
A=ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_A.so && \
bash tools/ab_env.sh r04ag_ab "DP_MI355X_LIB=$A" "DP_X=1"
