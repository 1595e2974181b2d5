#!/bin/bash
# persistent patch-conv engine: parity, then alone timings vs one workgroup per tile (debug 1 << 24)
set -o pipefail
mkdir -p gpurun_out/r05ae
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "patch_conv" > gpurun_out/r05ae/tests.log 2>&1 || { tail -30 gpurun_out/r05ae/tests.log; exit 1; }
tail -3 gpurun_out/r05ae/tests.log
for r in 1 2; do
  for d in 0 16777216; do
    echo "== dbg $d" >> gpurun_out/r05ae/alone.txt
    timeout -k 10 120 python -u tools/gemm_bench.py --only "768^2" --tile cv3_256x256 --dbg $d --iters 30 >> gpurun_out/r05ae/alone.txt 2>&1 || exit 1
    timeout -k 10 120 python -u tools/gemm_bench.py --only "rb conv 384" --tile cv3_192x256 --dbg $d --iters 30 >> gpurun_out/r05ae/alone.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r05ae/alone.txt
