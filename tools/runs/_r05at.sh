#!/bin/bash
# patch-conv: no priority changes (debug 1024) vs per-MFMA-run priority, stamped, alternating
set -o pipefail
mkdir -p gpurun_out/r05at
for r in 1 2; do
  for a in 0 1024; do
    timeout -k 10 100 python -u tools/cv3_stamps.py --size 768 --abl $a > gpurun_out/r05at/s768_$a.$r.log 2>&1 || exit 1
    timeout -k 10 100 python -u tools/cv3_stamps.py --size 384 --th 12 --abl $a > gpurun_out/r05at/s384_$a.$r.log 2>&1 || exit 1
  done
done
grep -H "per launch\|K loop per step" gpurun_out/r05at/*.log
