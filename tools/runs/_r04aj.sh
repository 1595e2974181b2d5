#!/bin/bash
# attention by sequence length at about equal work: where the fixed per-block costs go
set -o pipefail
mkdir -p gpurun_out/r04aj
for c in "35 577" "9 1152" "2 2304" "35 576" "1 4608"; do
  set -- $c
  timeout -k 10 120 python3 tools/attn_bench.py --quick --log2q --batch $1 --seq $2 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r04aj/attn_seq.txt || exit 1
done
