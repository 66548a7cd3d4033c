#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_migration.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mig_tests.log 2>&1 || { tail -40 gpurun_out/mig_tests.log; exit 1; }
tail -5 gpurun_out/mig_tests.log
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/bench_mig.json 2> gpurun_out/bench_mig.err || { tail -20 gpurun_out/bench_mig.err; exit 1; }
cat gpurun_out/bench_mig.json
