cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02v && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "forward_frame0 and mixed" -q --timeout 200 --timeout-method thread > gpurun_out/r02v/pytest.log 2>&1 && \
for g in 1 2 1 2; do DP_SIDE_STREAMS=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/r02v/b.json 2> gpurun_out/r02v/b.err || exit 1; echo "{\"ss\": $g, \"r\": $(cat gpurun_out/r02v/b.json)}" >> gpurun_out/r02v/all.jsonl; done
