#!/bin/bash
# attention half-tile software pipeline (variant B, 2 workgroups / CU) vs the product kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04ak && mkdir -p $O && \
B=ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_attnB.so && \
DP_MI355X_LIB=$B timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "attention" > $O/pytest_attn_B.log 2>&1 && \
for r in 1 2; do
  for c in "35 577" "9 1152"; do set -- $c
    timeout -k 10 120 python -u tools/attn_bench.py --quick --log2q --batch $1 --seq $2 2>&1 | grep -v amdgpu.ids >> $O/attn_A.txt && \
    DP_MI355X_LIB=$B timeout -k 10 120 python -u tools/attn_bench.py --quick --log2q --batch $1 --seq $2 2>&1 | grep -v amdgpu.ids >> $O/attn_B.txt || exit 1
  done
done
