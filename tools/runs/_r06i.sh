#!/bin/bash
# round 6 (i): why fc1's per-tile K loop is 1.33x qkv's on the same persistent engine -- stamps of
# the fc1 shape without GELU, the qkv shape with it, fc1 on 8- / 2-row tile bands (timing build)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i; mkdir -p $O
for R in 1 2; do
  DP_MI355X_LIB=$GRAFT_REPO_ROOT/ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_stamps.so \
    timeout -k 10 200 python -u tools/p8ph_stamps.py --more 2>/dev/null >> $O/p8ph_stamps.txt
done
