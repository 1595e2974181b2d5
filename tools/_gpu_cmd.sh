cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z8 && mkdir -p $O && \
for T in 8 0 8 0; do DP_CONV768_TILE=$T timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"tile\": $T, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done && \
for T in 8 0; do echo "tile=$T" >> $O/tl.txt; DP_CONV768_TILE=$T timeout -k 10 300 python -u tools/frame_timeline.py >> $O/tl.txt 2>&1 || exit 1; done
