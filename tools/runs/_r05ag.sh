#!/bin/bash
# the decoder's 1024 -> 256 3x3 convs (48^2, 96^2): every engine alone
set -o pipefail
mkdir -p gpurun_out/r05ag
timeout -k 10 300 python -u tools/gemm_bench.py --only "proj conv" --iters 30 > gpurun_out/r05ag/proj_conv.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05ag/proj_conv.txt
