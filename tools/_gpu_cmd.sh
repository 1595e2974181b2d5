cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02aa && \
timeout -k 10 300 python -u tools/gemm_bench.py --only "conv3x3 768" --tile big256x256,pbig256x256 > gpurun_out/r02aa/g.txt 2>&1 ; \
for g in 0 1024 0 1024 0 1024; do DP_GEMM_DEBUG=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/r02aa/b.json 2> gpurun_out/r02aa/b.err || exit 1; echo "{\"dbg\": $g, \"r\": $(cat gpurun_out/r02aa/b.json)}" >> gpurun_out/r02aa/all.jsonl; done
