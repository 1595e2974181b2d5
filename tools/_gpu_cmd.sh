cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r02k && mkdir -p $O && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "residual_layernorm or layernorm or tile_queues" --timeout 120 --timeout-method thread > $O/t_ln.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/t_model.log 2>&1 && \
for L in 1 0 1 0; do DP_LN_FUSE=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $O/b.json 2> $O/b.err || exit 1; echo "{\"ln\": $L, \"r\": $(cat $O/b.json)}" >> $O/all.jsonl; done && \
for L in 1 0; do DP_LN_FUSE=$L timeout -k 10 300 python -u tools/frame_shapes.py --top 14 >> $O/shapes.txt 2>&1 || exit 1; done
