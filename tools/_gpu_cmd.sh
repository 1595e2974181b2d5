cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r03f && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile 8ph256x256,dual256x128 --only fc1 > $O/gb_dual0.txt 2>&1 && \
for S in 3 6 9; do timeout -k 10 300 python -u tools/gemm_bench.py --tile dual256x128 --only fc1 --dbg $(( (1<<21) + (S<<24) )) > $O/gb_dual_s$S.txt 2>&1 || exit 1; done && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile dual256x128 --only qkv > $O/gb_dual_qkv.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile dual256x128 --only qkv --dbg $(( (1<<21) + (6<<24) )) > $O/gb_dual_qkv_s6.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/bench.json 2> $O/bench.err && \
cd $GRAFT_REPO_ROOT && DP_MI355X_LIB=$GRAFT_REPO_ROOT/ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_attnexp.so timeout -k 10 300 python -u tools/attn_bench.py --ablate > gpurun_out/r03f/attn_ablate.txt 2>&1
