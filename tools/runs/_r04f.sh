cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04f && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -v -s --timeout 300 --timeout-method thread -k "concurrent_schedule" > $O/pytest_sched.log 2>&1 && \
bash tools/ab_env.sh r04f_ab "DP_SIDE_GATE=0" "DP_SIDE_GATE=fc2:fc1" "DP_SIDE_GATE=fc2:proj" "DP_SIDE_GATE=qkv:fc1"
