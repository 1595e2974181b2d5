#!/bin/bash
# round 6 (d): fc1 / qkv per-tile stamps (timing build), serial-frame kernel trace (frame budget +
# per-kernel alone times) of the current tree
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
DP_MI355X_LIB=$GRAFT_REPO_ROOT/ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_stamps.so \
  timeout -k 10 200 python -u tools/p8ph_stamps.py > $O/p8ph_stamps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o prof --output-format csv \
  -- python3 tools/frame_once.py --frames 5 --serial > $O/prof_serial.log 2>&1
python3 tools/frame_budget.py $O/prof_serial/prof_kernel_trace.csv --md $O/frame_budget.md --alone-md $O/kernel_alone.md > /dev/null
