#!/bin/bash
# where the 1536^2 loop's submitting thread spends its time
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ar && mkdir -p $O && \
timeout -k 10 300 python -u tools/loop_bench.py --frames 96 --trace 2>&1 | grep '^{' >> $O/loop.jsonl && \
timeout -k 10 300 python -u tools/loop_bench.py --frames 96 2>&1 | grep '^{' >> $O/loop.jsonl
