#!/bin/bash
# A/B of the consecutive-bin layout and the one-exp-per-lane sweep (sweep8_near): parity tests
# on lib_en, then config 3 at full length and short runs of configs 4 / 2 / 5 for every
# abtest/lib_*.so (lib_base = HEAD, lib_lay = layout only, lib_en = layout + sweep8_near).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FITOCT_LIB_PATH=$PWD/abtest/lib_en.so timeout -k 10 400 python -u -m pytest tests/test_gpu_logp.py tests/test_gpu_sampler.py tests/test_gpu_spec.py tests/test_gpu_migration.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/ab_en_tests.log 2>&1 || { tail -30 gpurun_out/ab_en_tests.log; exit 1; }
tail -2 gpurun_out/ab_en_tests.log
timeout -k 10 500 bash scripts/ab_full3.sh > gpurun_out/ab_en_full3.txt 2>&1 || { cat gpurun_out/ab_en_full3.txt; exit 1; }
cat gpurun_out/ab_en_full3.txt
AB_CONFIGS="4 2 5" timeout -k 10 500 bash scripts/ab_libs.sh > gpurun_out/ab_en_short.txt 2>&1 || { cat gpurun_out/ab_en_short.txt; exit 1; }
cat gpurun_out/ab_en_short.txt
