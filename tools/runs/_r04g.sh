cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04g && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -s --timeout 300 --timeout-method thread -k "attention" > $O/pytest_attn.log 2>&1 && \
A=ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_attnA.so && \
for r in 1 2 3; do
  DP_MI355X_LIB=$A timeout -k 10 120 python -u tools/attn_bench.py --quick --log2q >> $O/attn_A.txt 2>&1 && \
  timeout -k 10 120 python -u tools/attn_bench.py --quick --log2q >> $O/attn_B.txt 2>&1 || exit 1
done && \
bash tools/ab_env.sh r04g_ab "DP_MI355X_LIB=$A" "DP_X=1"
