cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02u && \
for g in 1 4 2 1 4 2; do DP_SIDE_SPLITK=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/r02u/b.json 2> gpurun_out/r02u/b.err || exit 1; echo "{\"sk\": $g, \"r\": $(cat gpurun_out/r02u/b.json)}" >> gpurun_out/r02u/all.jsonl; done
