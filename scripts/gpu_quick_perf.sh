#!/bin/bash
# Sampler parity tests + short perf lines for configs 3, 5, 2 (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/qp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_logp.py tests/test_gpu_smoke.py tests/test_gpu_migration.py tests/test_gpu_batch.py tests/test_gpu_genquant.py -x -q --timeout 300 --timeout-method thread > gpurun_out/qp/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/qp/tests.log | head -20; tail -20 gpurun_out/qp/tests.log; exit 1; }
tail -1 gpurun_out/qp/tests.log
for c in 3 5 2 4; do
  it="200,200"; [ $c = 5 ] && it="100,100"
  timeout -k 10 200 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --iters $it > gpurun_out/qp/c$c.json 2>gpurun_out/qp/err || { tail gpurun_out/qp/err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/qp/c$c.json'));print('config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
