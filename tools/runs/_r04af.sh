cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04af && mkdir -p $O && \
for r in 1 2 3; do timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_$r.json 2> $O/bench_$r.err || exit 1; done && \
timeout -k 10 400 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err
