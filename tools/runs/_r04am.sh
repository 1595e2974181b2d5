#!/bin/bash
# 4K --pointcloud video loop: zero-copy PLY body write vs the round-4 bytes copy, 24 frames, alternated
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04am && mkdir -p $O && \
for r in 1 2; do
  timeout -k 10 300 python -u tools/loop_bench.py --frames 24 --size 3840x2160 --pointcloud 2>&1 | grep -v amdgpu.ids >> $O/loop_A.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 24 --size 3840x2160 --pointcloud --ply-copy 2>&1 | grep -v amdgpu.ids >> $O/loop_B.jsonl || exit 1
done
