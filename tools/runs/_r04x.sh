cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04x && mkdir -p $O && \
for r in 1 2; do for sq in 577 576 640 512 1024; do timeout -k 10 120 python -u tools/attn_bench.py --quick --log2q --seq $sq >> $O/attn_seq.txt 2>&1 || exit 1; done; done
