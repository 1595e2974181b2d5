cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04y && mkdir -p $O && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "deconv" --tile auto,p8ph256x256,big256x256,sk256x256 --ablate > $O/deconv.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "conv3x3 384" --tile auto,big320x256,cv3_256x256,pbig320x256 > $O/conv384.txt 2>&1
