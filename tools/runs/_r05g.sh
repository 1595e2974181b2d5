#!/bin/bash
# round 5 (g): the latent project / upsample chains beside the patch encoder (DP_LAT_EARLY=1): capture check,
# schedule test, A/B
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05g
DP_LAT_EARLY=1 timeout -k 10 200 python -u -X faulthandler tools/dbg_sched.py > gpurun_out/r05g/dbg.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "concurrent_schedule" > gpurun_out/r05g/pytest.log 2>&1
bash tools/ab_env.sh r05g "DP_LAT_EARLY=0" "DP_LAT_EARLY=1"
