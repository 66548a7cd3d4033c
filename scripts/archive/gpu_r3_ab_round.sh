#!/bin/bash
# A/B bundle for latency-only / layout changes: bitwise draws of every abtest/lib_*.so vs
# lib_base.so, config-3 L2->memory writes per library, config 3 at full length, short runs
# of configs 4, 2, 5.  Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/ab_bitwise.py > gpurun_out/ab_bitwise.txt 2>&1 || { cat gpurun_out/ab_bitwise.txt; exit 1; }
cat gpurun_out/ab_bitwise.txt
timeout -k 10 600 bash scripts/pmc_write_ab.sh > gpurun_out/ab_pmcw.txt 2>&1 || { cat gpurun_out/ab_pmcw.txt; exit 1; }
cat gpurun_out/ab_pmcw.txt
timeout -k 10 400 bash scripts/ab_full3.sh > gpurun_out/ab_full3.txt 2>&1 || { cat gpurun_out/ab_full3.txt; exit 1; }
cat gpurun_out/ab_full3.txt
AB_CONFIGS="${AB_SHORT:-4 2 5}" timeout -k 10 500 bash scripts/ab_libs.sh > gpurun_out/ab_short.txt 2>&1 || { cat gpurun_out/ab_short.txt; exit 1; }
cat gpurun_out/ab_short.txt
