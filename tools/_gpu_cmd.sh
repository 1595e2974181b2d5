bash tools/gpu_check.sh r02d tests smoke bench prof
