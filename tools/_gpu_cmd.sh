cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z11 && mkdir -p $O && \
for S in 1 0 1 0; do DP_SIDE_SYNC=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"sync\": $S, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
