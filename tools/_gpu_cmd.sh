cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z9 && mkdir -p $O && \
for T in 8 0 8 0; do DP_QKV_TILE=$T timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"tile\": $T, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
