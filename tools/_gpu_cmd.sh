cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r01zc && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01zc/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r01zc/bench.json 2> gpurun_out/r01zc/bench.err && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r01zc/smoke.log 2>&1
