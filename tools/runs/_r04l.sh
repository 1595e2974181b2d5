cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04l && mkdir -p $O && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "rb conv" --tile auto,big256x256,sk256x256,big256x128,big320x256 > $O/rb.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "proj conv" --tile auto,big256x256,sk256x256 > $O/projconv.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "conv3x3" --tile auto,big256x256,sk256x256 > $O/conv.txt 2>&1
