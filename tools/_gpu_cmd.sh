cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02w && mkdir -p $O && \
for F in -1 8 16 23 -1 8 16 23; do DP_FOV_AT=$F timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"fov_at\": $F, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
