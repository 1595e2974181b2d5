#!/bin/bash
# One bounded GPU session (run on the gpurun box from the repo root):
#   GPU tests -> bench line -> rocprofv3 kernel-trace stats -> FETCH/WRITE PMC passes.
# Every GPU step has its own time limit; the first failure ends the script.
# Usage: tools/gpu_check.sh <tag> [tests|smoke|bench|prof|pmc|sq|serial|side|loop ...]   (default: tests bench prof pmc)
set -eo pipefail
TAG=${1:-r01}
shift || true
STEPS=${*:-tests bench prof pmc}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
for S in $STEPS; do
  case $S in
    tests)
      DP_TEST_METRICS=$OUT/test_metrics.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof --output-format csv \
        -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 ;;
    pmc)
      # separate passes (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2); eager forward so every dispatch is attributed
      timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc \
        -- python3 tools/frame_once.py > $OUT/pmc_fetch.log 2>&1
      timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc \
        -- python3 tools/frame_once.py > $OUT/pmc_write.log 2>&1 ;;
    sq)
      # SQ wave-state / MFMA-busy passes over an eager forward (tools/pmc_sq.py), one pass each
      timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv \
        -d $OUT/pmc_sq1 -o pmc -- python3 tools/frame_once.py > $OUT/pmc_sq1.log 2>&1
      timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv \
        -d $OUT/pmc_sq2 -o pmc -- python3 tools/frame_once.py > $OUT/pmc_sq2.log 2>&1 ;;
    gemm)
      # GEMM engine micro-benchmarks: fc1 / sq4096 on the 8-phase and dual engines, with the no-store ablation
      timeout -k 10 300 python -u tools/gemm_bench.py --tile 8ph256x256,dual256x128,big320x256 --only fc1 --ablate \
        > $OUT/gemm_fc1.txt 2>&1
      timeout -k 10 300 python -u tools/gemm_bench.py --tile 8ph256x256,big320x256 --only sq4096 --ablate \
        > $OUT/gemm_sq4096.txt 2>&1
      timeout -k 10 300 python -u tools/gemm_bench.py --tile big320x256,8ph256x256 --only + --ablate \
        > $OUT/gemm_res.txt 2>&1 ;;
    fc1)
      # fc1 on the three engines that can run it, same box
      timeout -k 10 300 python -u tools/gemm_bench.py --tile 8ph256x256,p8ph256x256,8ph320x256 --only fc1 --ablate \
        > $OUT/gemm_fc1_engines.txt 2>&1 ;;
    serial)
      # serial frames (every launch alone on the chip): the per-frame budget and per-kernel alone times
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o prof --output-format csv \
        -- python3 tools/frame_once.py --frames 5 --serial > $OUT/prof_serial.log 2>&1
      python3 tools/frame_budget.py $OUT/prof_serial/prof_kernel_trace.csv --md $OUT/frame_budget.md \
        --alone-md $OUT/kernel_alone.md > /dev/null ;;
    side)
      # side-encoder cost by ablation (DP_ABLATE=side: image / FOV encoders skipped) vs the full frame
      DP_ABLATE=side timeout -k 10 300 python -u bench.py --ab --no-cpu-baseline --steps 40 > $OUT/bench_noside.json 2> $OUT/bench_noside.err
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 > $OUT/bench_side.json 2> $OUT/bench_side.err ;;
    loop)
      # the video loop as users run it (configs 3 and 5): PNG frames -> GPU -> PNG (+ PLY)
      timeout -k 10 400 python -u tools/loop_bench.py --frames 64 --size 1536x1536 > $OUT/loop_1536.log 2>&1
      timeout -k 10 400 python -u tools/loop_bench.py --frames 64 --size 3840x2160 --pointcloud > $OUT/loop_4k_pc.log 2>&1 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
  echo "step $S ok"
done
