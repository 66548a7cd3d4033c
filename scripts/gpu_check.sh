#!/bin/bash
# GPU test suite + one headline bench step (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
