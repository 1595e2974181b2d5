cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z6 && mkdir -p $O && \
DP_ATTN_NST=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention and True" --timeout 120 --timeout-method thread > $O/t_attn.log 2>&1 && \
for N in 3 2 3 2; do echo "nst=$N" >> $O/attn.txt; DP_ATTN_NST=$N DP_ATTN_LOG2Q=1 timeout -k 10 120 python -u tools/attn_bench.py --quick >> $O/attn.txt 2>&1 || exit 1; done && \
for N in 3 2 3 2; do DP_ATTN_NST=$N timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"nst\": $N, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
