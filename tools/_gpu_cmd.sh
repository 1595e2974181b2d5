cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02l && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k attention --timeout 120 --timeout-method thread > $O/t_attn.log 2>&1 && \
for P in 1 0 1 0; do echo "pf=$P" >> $O/attn.txt; DP_ATTN_PF=$P timeout -k 10 120 python -u tools/attn_bench.py --quick >> $O/attn.txt 2>&1 || exit 1; done && \
timeout -k 10 200 python -u tools/attn_bench.py >> $O/attn_full.txt 2>&1 && \
for P in 1 0 1 0; do DP_ATTN_PF=$P timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"pf\": $P, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/t_model.log 2>&1
