#!/bin/bash
# fexp with three-VGPR v_fma_f64 (no coefficient copy per Horner step): bitwise draws vs
# lib_base, config 3 at full length, short runs of configs 2, 5, 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/ab_bitwise.py > gpurun_out/fmav_bitwise.txt 2>&1 || { cat gpurun_out/fmav_bitwise.txt; exit 1; }
grep -v amdgpu gpurun_out/fmav_bitwise.txt
timeout -k 10 400 bash scripts/ab_full3.sh > gpurun_out/fmav_full3.txt 2>&1 || { cat gpurun_out/fmav_full3.txt; exit 1; }
cat gpurun_out/fmav_full3.txt
AB_CONFIGS="2 5 4" timeout -k 10 600 bash scripts/ab_libs.sh > gpurun_out/fmav_short.txt 2>&1 || { cat gpurun_out/fmav_short.txt; exit 1; }
cat gpurun_out/fmav_short.txt
