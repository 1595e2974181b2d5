cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02y && \
for g in 0 1 7 11 0 1 7 11; do DP_SIDE_TILE=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/r02y/b.json 2> gpurun_out/r02y/b.err || exit 1; echo "{\"t\": $g, \"r\": $(cat gpurun_out/r02y/b.json)}" >> gpurun_out/r02y/all.jsonl; done
