cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z10 && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread -k "decoder_streams or pipeline or graph_replays" > $O/t_model.log 2>&1
