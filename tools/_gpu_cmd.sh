cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r01r && \
timeout -k 10 400 python -u -m pytest tests/test_pointcloud.py tests/test_frameloop.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r01r/pytest_pc.log 2>&1
