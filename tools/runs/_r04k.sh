cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04k && mkdir -p $O && \
timeout -k 10 400 python -u bench.py > $O/bench1.json 2> $O/bench1.err && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 40 > $O/bench2.json 2> $O/bench2.err
