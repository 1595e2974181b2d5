cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02y && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/t_model.log 2>&1 && \
for S in 1 0 1 0; do DP_LAT0_SK=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"lat0sk\": $S, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
