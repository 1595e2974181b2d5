cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02m && mkdir -p $O && \
for T in 0 12 4 0 12 4; do DP_SIDE_TILE=$T timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"side_tile\": $T, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
