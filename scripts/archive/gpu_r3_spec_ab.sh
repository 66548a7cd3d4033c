set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_migration.py tests/test_gpu_warm_restart.py tests/test_gpu_multidevice.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r3_spec.log 2>&1 || exit 1
AB_DIR=abtest/c4 AB_CONFIGS=4 timeout -k 10 400 bash scripts/ab_libs.sh > gpurun_out/r3_ab_c4.txt 2>&1 || exit 1
AB_DIR=abtest/spec timeout -k 10 500 bash scripts/ab_full3.sh > gpurun_out/r3_ab_spec_c3.txt 2>&1 || exit 1
AB_DIR=abtest/spec AB_CONFIGS="5 2" timeout -k 10 500 bash scripts/ab_libs.sh > gpurun_out/r3_ab_spec_c52.txt 2>&1 || exit 1
