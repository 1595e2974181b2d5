#!/bin/bash
# the 4K --pointcloud loop over 64 frames (steady state beyond the pipeline's fill and drain)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04aq && mkdir -p $O && \
timeout -k 10 400 python -u tools/loop_bench.py --frames 64 --size 3840x2160 --pointcloud 2>&1 | grep '^{' >> $O/loop_4k.jsonl && \
timeout -k 10 400 python -u tools/loop_bench.py --frames 64 --size 3840x2160 --pointcloud --workers 12 2>&1 | grep '^{' >> $O/loop_4k.jsonl
