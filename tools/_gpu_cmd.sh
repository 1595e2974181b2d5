cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02i && mkdir -p $O && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "persistent" --timeout 120 --timeout-method thread > $O/t_pbig.log 2>&1 && \
for D in 0 4096 12288 20480 0 4096 12288 20480; do DP_GEMM_DEBUG=$D timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"dbg\": $D, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done && \
for D in 0 4096 12288 20480; do DP_GEMM_DEBUG=$D timeout -k 10 300 python -u tools/frame_shapes.py --dbg $D --top 12 >> $O/shapes.txt 2>&1 || exit 1; done
