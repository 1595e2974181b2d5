cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02q && \
DP_ATTN_SB=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -q --timeout 200 --timeout-method thread > gpurun_out/r02q/pytest.log 2>&1 && \
for v in 1 2 1 2; do DP_ATTN_SB=$v timeout -k 10 300 python -u tools/attn_bench.py --quick >> gpurun_out/r02q/attn_$v.txt 2>&1 || exit 1; done
