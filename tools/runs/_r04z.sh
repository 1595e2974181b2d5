cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04z && mkdir -p $O && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "384" --tile auto,big320x256,cv3_256x256 > $O/conv384.txt 2>&1 && \
bash tools/ab_env.sh r04z_ab "DP_X=0" "DP_GEMM_DEBUG=134217728"
