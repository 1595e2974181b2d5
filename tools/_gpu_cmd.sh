cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02j && \
DP_ATTN_VSUM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -q --timeout 200 --timeout-method thread > gpurun_out/r02j/pytest.log 2>&1 && \
for v in 0 1 0 1; do DP_ATTN_VSUM=$v timeout -k 10 300 python -u tools/attn_bench.py --quick >> gpurun_out/r02j/attn_$v.txt 2>&1 || exit 1; done
