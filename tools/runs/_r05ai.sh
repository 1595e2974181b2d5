#!/bin/bash
# the decoder's 48^2 / 96^2 / 192^2 ResidualBlock convs alone: planner's engine vs split-K
set -o pipefail
mkdir -p gpurun_out/r05ai
for s in "rb conv 48" "rb conv 96" "rb conv 192" "conv3x3 48" "conv3x3 96"; do
  timeout -k 10 120 python -u tools/gemm_bench.py --only "$s" --tile auto,splitk256x256,sk256x256,big256x128 --iters 30 >> gpurun_out/r05ai/rb_small.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r05ai/rb_small.txt
