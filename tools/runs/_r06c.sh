#!/bin/bash
# round 6 (c): 3x3 patch-conv K loop with constant-offset LDS addressing (unrolled taps, tight patch
# buffers, scalar-base weight DMA, buffer-resource patch DMA) -- correctness, alone times vs the HEAD
# library (ab_old/), in-frame A/B, then the GPU tests + bench
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
NEW=$GRAFT_REPO_ROOT/ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x.so
OLD=$GRAFT_REPO_ROOT/ab_old/libdp_mi355x.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "cv3 or patch_conv or head or conv" --timeout 120 --timeout-method thread > $O/pytest_cv3.log 2>&1
for L in OLD NEW OLD NEW; do
  eval LIB=\$$L
  for A in "--size 768 --no-res" "--size 768" "--size 384 --th 12"; do
    echo "$L $A: $(DP_MI355X_LIB=$LIB timeout -k 10 120 python -u tools/cv3_stamps.py $A --seconds 1.5 2>/dev/null | grep plain)" >> $O/cv3_alone.txt
  done
done
for R in 1 2; do for L in OLD NEW; do
  eval LIB=\$$L
  DP_MI355X_LIB=$LIB timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err
done; done
python3 - <<'PY' > $O/ab.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/r06c/ab_*.json")):
    d = json.load(open(f)); print(f, d.get("value"), d.get("ms_per_step"), (d.get("parity") or {}).get("depth_rel_l1"))
PY
bash tools/gpu_check.sh r06c tests
