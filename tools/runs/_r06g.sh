#!/bin/bash
# round 6 (g): 8-phase 320 x 256 engine, A pieces of step s+2 spread over phases 1-3 (1 + 2 + 2)
# -- GEMM tests, proj / fc2 alone vs the HEAD library (ab_old/), in-frame A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g; mkdir -p $O
NEW=$GRAFT_REPO_ROOT/ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x.so
OLD=$GRAFT_REPO_ROOT/ab_old/libdp_mi355x.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "8phase or 8ph320 or ln_consumer or ln_producer or split_residual" --timeout 120 --timeout-method thread > $O/pytest_p8.log 2>&1
for L in OLD NEW OLD NEW; do
  eval LIB=\$$L
  DP_MI355X_LIB=$LIB timeout -k 10 200 python -u tools/gemm_bench.py --tile 8ph320x256 --only "+res" 2>/dev/null | sed "s/^/$L /" >> $O/res_alone.txt
done
for R in 1 2; do for L in OLD NEW; do
  eval LIB=\$$L
  DP_MI355X_LIB=$LIB timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/ab_${L}_$R.json 2> $O/ab_${L}_$R.err
done; done
python3 - <<'PY' > $O/ab.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/r06g/ab_*.json")):
    d = json.load(open(f)); print(f, d.get("value"), d.get("ms_per_step"), (d.get("parity") or {}).get("depth_rel_l1"))
PY
