#!/bin/bash
# Deep speculation A/B: speculative-path GPU tests on the default library, bitwise draws of
# abtest/lib_deep.so vs lib_base.so (FITOCT_DEEP_SPEC=0), then config 2 / 5 short-run rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r3_deep_spec.log 2>&1 || { tail -20 gpurun_out/r3_deep_spec.log; exit 1; }
timeout -k 10 400 python3 -u scripts/ab_bitwise.py > gpurun_out/r3_deep_bitwise.txt 2>&1 || { cat gpurun_out/r3_deep_bitwise.txt; exit 1; }
AB_CONFIGS="2" timeout -k 10 500 bash scripts/ab_libs.sh > gpurun_out/r3_deep_ab.txt 2>&1 || exit 1
cat gpurun_out/r3_deep_bitwise.txt gpurun_out/r3_deep_ab.txt
