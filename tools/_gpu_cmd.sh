bash tools/gpu_check.sh r02f sq pmc
