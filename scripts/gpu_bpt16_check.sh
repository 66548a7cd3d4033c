set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_logp.py tests/test_gpu_sampler.py -x -v --timeout 300 --timeout-method thread -k "N4096 or N3001 or N2049 or N8192 or lasso-N3001 or lasso-N200 or horseshoe-N2048" > gpurun_out/bpt16.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/bpt16.log | head; tail -30 gpurun_out/bpt16.log; exit 1; }
grep -E "PASSED|passed" gpurun_out/bpt16.log | tail -12
CONFIGS=4 bash scripts/gpu_configs.sh
