cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04u && mkdir -p $O && \
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -k "loop or config5 or depth_pro_run or frameloop or config1" > $O/pytest_loop.log 2>&1 && \
timeout -k 10 400 python -u tools/loop_bench.py --frames 64 --size 1536x1536 > $O/loop_1536.log 2>&1 && \
timeout -k 10 400 python -u tools/loop_bench.py --frames 8 --size 3840x2160 --pointcloud > $O/loop_4k_pc.log 2>&1
