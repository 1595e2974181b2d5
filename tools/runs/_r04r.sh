cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04r && mkdir -p $O && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "proj+res" --tile 8ph320x256,dual256x128,big320x256,big256x128 > $O/proj.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "fc2+res" --tile 8ph320x256,dual256x128,big320x256 > $O/fc2.txt 2>&1 && \
DP_GEMM_DEBUG=2097152 timeout -k 10 300 python -u tools/gemm_bench.py --only "proj+res" --tile dual256x128 > $O/proj_stagger.txt 2>&1
