cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04m && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_abi.py -v -s --timeout 300 --timeout-method thread -k "split_k or stream_k or plan or every_big" > $O/pytest_splitk.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -v -s --timeout 300 --timeout-method thread -k "forward_frame0 or stages" > $O/pytest_model.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "rb conv" --tile auto,big256x256,big256x128 > $O/rb.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "proj conv" --tile auto,sk256x256 > $O/projconv.txt 2>&1 && \
bash tools/ab_env.sh r04m_ab "DP_X=0" "DP_GEMM_DEBUG=134217728"
