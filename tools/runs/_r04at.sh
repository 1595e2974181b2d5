#!/bin/bash
# frame uploads / downloads on copy streams vs on the compute stream: 1536^2 (96 frames) and
# 4K --pointcloud (48 frames) loops, alternated, after the frame-loop GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04at && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_frameloop.py tests/test_gpu_configs.py tests/test_pointcloud.py -x -v --timeout 120 --timeout-method thread > $O/pytest_loop.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u tools/loop_bench.py --frames 96 2>&1 | grep '^{' >> $O/loop_1536.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 96 --no-copy-streams 2>&1 | grep '^{' >> $O/loop_1536.jsonl || exit 1
done && \
timeout -k 10 400 python -u tools/loop_bench.py --frames 48 --size 3840x2160 --pointcloud 2>&1 | grep '^{' >> $O/loop_4k.jsonl && \
timeout -k 10 400 python -u tools/loop_bench.py --frames 48 --size 3840x2160 --pointcloud --no-copy-streams 2>&1 | grep '^{' >> $O/loop_4k.jsonl
