#!/bin/bash
# ln_merge pre-pass on 64-thread workgroups (variant B) vs 256: kernel durations + in-frame A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04av && mkdir -p $O && \
B=ml-depth-pro-video_amd/depth_pro/_lib/libdp_mi355x_lnmB.so && \
DP_MI355X_LIB=$B timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "ln" > $O/pytest_ln_B.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profA -o prof --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/profA.log 2>&1 && \
DP_MI355X_LIB=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profB -o prof --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/profB.log 2>&1 && \
bash tools/ab_env.sh r04av_ab "DP_MI355X_LIB=$B" "DP_X=1"
