cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r03b && mkdir -p $O && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> $O/pytest_gpu.log; \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile dual256x128,8ph256x256 --ablate --only fc1 > $O/gb_fc1.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile dual256x128,big320x256 --ablate --only qkv > $O/gb_qkv.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile dual256x128,big320x256 --ablate --only res > $O/gb_res.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile dual256x128,pbig256x256 --ablate --only "768^2 256->256" > $O/gb_conv.txt 2>&1
