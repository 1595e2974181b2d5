#!/bin/bash
# PNG writer without GIL-held copies vs the copying one, in the 1536^2 and 4K --pointcloud loops
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ao && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_frameloop.py tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > $O/pytest_loop.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u tools/loop_bench.py --frames 64 2>&1 | grep '^{' >> $O/loop_1536_A.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 64 --png-copy 2>&1 | grep '^{' >> $O/loop_1536_B.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 24 --size 3840x2160 --pointcloud 2>&1 | grep '^{' >> $O/loop_4k_A.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 24 --size 3840x2160 --pointcloud --png-copy 2>&1 | grep '^{' >> $O/loop_4k_B.jsonl || exit 1
done
