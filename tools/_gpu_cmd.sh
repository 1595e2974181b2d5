cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02p && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k attention --timeout 120 --timeout-method thread > $O/t_attn.log 2>&1 && \
for A in 1 0 1 0; do DP_ATTN_SADD=$A timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"sadd\": $A, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
