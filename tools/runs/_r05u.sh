#!/bin/bash
# round 5 (u): profile set of the tree after qkv on the persistent engine, producer-merged LN stats,
# the early fusion-0 conv, the deconv store and the cv3 residual prefetch: tests, smoke, bench,
# rocprofv3 kernel stats, FETCH/WRITE + SQ PMC passes, side-encoder ablation
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh r05u tests smoke bench prof pmc sq side
