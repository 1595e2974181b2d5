cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ab && mkdir -p $O && \
timeout -k 10 300 python -u tools/cold_bench.py > $O/cold.txt 2>&1
