cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z12 && mkdir -p $O && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "border or head or conv3x3" --timeout 120 --timeout-method thread > $O/t_k.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/t_model.log 2>&1 && \
for S in 1 0 1 0; do DP_HEAD0_COMPOSE=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"h0c\": $S, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
