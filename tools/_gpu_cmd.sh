cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r03c && mkdir -p $O && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256 --only fc1 > $O/gb_fc1.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256 --only fc1 --dbg 1048576 > $O/gb_fc1_general.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile big320x256 --only qkv > $O/gb_qkv.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --tile big320x256 --only qkv --dbg 1048576 > $O/gb_qkv_general.txt 2>&1 ; \
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> $O/pytest_gpu.log
