cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02s && \
for g in 0 512 256 0 512 256; do DP_GEMM_DEBUG=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/r02s/b.json 2> gpurun_out/r02s/b.err || exit 1; echo "{\"dbg\": $g, \"r\": $(cat gpurun_out/r02s/b.json)}" >> gpurun_out/r02s/all.jsonl; done
