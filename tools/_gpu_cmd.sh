cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r03a && mkdir -p $O && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256,pbig256x256 --ablate --only fc1 > $O/gb_fc1.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256 --ablate --only sq4096 > $O/gb_sq.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256 --ablate --only qkv > $O/gb_qkv.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256 --ablate --only res > $O/gb_res.txt 2>&1 && \
timeout -k 10 400 python -u tools/gemm_bench.py --tile big256x256,pbig256x256,big320x256 --ablate --only "768^2 256->256" > $O/gb_conv.txt 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --torch-only > $O/gb_torch.txt 2>&1
