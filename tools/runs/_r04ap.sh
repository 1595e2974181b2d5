#!/bin/bash
# the GIL switch interval in the 1536^2 loop (default 5 ms vs 1 ms / 0.5 ms), alternated
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ap && mkdir -p $O && \
for r in 1 2; do
  timeout -k 10 300 python -u tools/loop_bench.py --frames 96 2>&1 | grep '^{' >> $O/loop.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 96 --switch-ms 1 2>&1 | grep '^{' >> $O/loop.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 96 --switch-ms 0.5 2>&1 | grep '^{' >> $O/loop.jsonl || exit 1
done
