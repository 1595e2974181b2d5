cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02c && \
for d in bf16 mixed fp16 mixed bf16; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --dtype $d --steps 40 > gpurun_out/r02c/bench_$d.json 2> gpurun_out/r02c/bench_$d.err || exit 1; cat gpurun_out/r02c/bench_$d.json >> gpurun_out/r02c/all.jsonl; done
