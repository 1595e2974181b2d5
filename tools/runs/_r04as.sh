#!/bin/bash
# kernel + memory-copy trace of the 1536^2 video loop: per-frame GPU busy time, gaps and copies
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04as && mkdir -p $O && \
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o loop --output-format csv -- python3 -u tools/loop_bench.py --frames 48 > $O/loop.log 2>&1
