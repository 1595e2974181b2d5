cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ah && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread -k "attention" > $O/pytest_attn.log 2>&1
