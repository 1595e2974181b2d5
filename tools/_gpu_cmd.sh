cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02p && \
DP_SIDE_MODE=serial timeout -k 10 300 python -u tools/parity_probe.py > gpurun_out/r02p/serial.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02p/pytest_gpu.log 2>&1
