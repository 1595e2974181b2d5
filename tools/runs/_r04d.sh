cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04d && mkdir -p $O && \
DP_LN_FOLD=1 timeout -k 10 300 python -u tools/frame_shapes.py --top 40 > $O/shapes_fold.txt 2>&1 && \
DP_LN_FOLD=0 timeout -k 10 300 python -u tools/frame_shapes.py --top 40 > $O/shapes_nofold.txt 2>&1 && \
DP_LN_FOLD=1 timeout -k 10 300 python -u tools/frame_shapes.py --top 40 --dbg 33554432 > $O/shapes_fold_fc1_8ph320.txt 2>&1 && \
DP_LN_FOLD=1 timeout -k 10 300 python -u tools/frame_streams.py > $O/streams_fold.txt 2>&1 && \
DP_LN_FOLD=0 timeout -k 10 300 python -u tools/frame_streams.py > $O/streams_nofold.txt 2>&1
