cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04e && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -v -s --timeout 300 --timeout-method thread -k "concurrent_schedule or bicubic or forward_frame0" > $O/pytest_sched.log 2>&1 && \
bash tools/ab_env.sh r04e_ab "DP_SIDE_GATE=0" "DP_SIDE_GATE=1" "DP_SIDE_GATE=1 DP_LN_FOLD=0" "DP_SIDE_GATE=0 DP_LN_FOLD=0"
