#!/bin/bash
# PLY vertex records interleaved on the GPU vs on the host (numpy) in the 4K --pointcloud loop,
# after the point-cloud / frame-loop GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04an && mkdir -p $O && \
timeout -k 10 300 python -u -m pytest tests/test_pointcloud.py tests/test_frameloop.py tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > $O/pytest_pc.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u tools/loop_bench.py --frames 24 --size 3840x2160 --pointcloud 2>&1 | grep -v amdgpu.ids | grep '^{' >> $O/loop_A.jsonl && \
  timeout -k 10 300 python -u tools/loop_bench.py --frames 24 --size 3840x2160 --pointcloud --ply-host 2>&1 | grep -v amdgpu.ids | grep '^{' >> $O/loop_B.jsonl || exit 1
done
