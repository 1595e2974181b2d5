cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r01t && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread -s > gpurun_out/r01t/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --only head --tile big256x128,big512x128 > gpurun_out/r01t/head.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r01t/bench.json 2> gpurun_out/r01t/bench.err
