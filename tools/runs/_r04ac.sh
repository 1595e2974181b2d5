cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ac && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -v -s --timeout 300 --timeout-method thread -k "concurrent_schedule or forward_frame0 or graph" > $O/pytest_pf.log 2>&1 && \
bash tools/ab_env.sh r04ac_ab "DP_PREFETCH=1" "DP_PREFETCH=0"
