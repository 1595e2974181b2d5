cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r01u && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r01u/pytest_model.log 2>&1 && \
for i in 1 2; do for F in 1 0; do DP_FOV_LATE=$F timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/fov_late=$F /" >> gpurun_out/r01u/ab.log || exit 1; done; done
