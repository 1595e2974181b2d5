cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02z4 && mkdir -p $O && \
for S in "0 4" "1 4" "0 8" "1 8" "0 16" "1 16"; do set -- $S; GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --pipeline $1 > $O/b.json 2> $O/b.err || exit 1; echo "{\"pipe\": $1, \"q\": $2, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done
