cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r01p && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread -s > gpurun_out/r01p/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r01p/bench.json 2> gpurun_out/r01p/bench.err && \
timeout -k 10 300 python -u tools/gemm_bench.py --only conv > gpurun_out/r01p/gemm_conv.log 2>&1
