set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 300 --timeout-method thread > gpurun_out/batch_tests.log 2>&1 || { tail -40 gpurun_out/batch_tests.log; exit 1; }
tail -8 gpurun_out/batch_tests.log
CONFIGS=5 bash scripts/gpu_configs.sh
