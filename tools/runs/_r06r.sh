#!/bin/bash
# round 6 (r): the clock the chip holds under fc1 with and without its GELU epilogue (GRBM_GUI_ACTIVE)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o pmc \
  -- python3 tools/gelu_clock.py > $O/pmc.log 2>&1
python3 tools/gelu_clock.py --report $O/pmc/pmc_counter_collection.csv $O/pmc/pmc_kernel_trace.csv > $O/gelu_clock.txt
