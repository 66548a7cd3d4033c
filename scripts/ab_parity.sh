#!/bin/bash
# Parity (logp + sampler horizon) for every ablib/lib_*.so, then the perf A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for l in ablib/lib_*.so; do
  n=$(basename $l .so)
  FITOCT_LIB_PATH=$PWD/$l timeout -k 10 300 python -u -m pytest tests/test_gpu_logp.py tests/test_gpu_sampler.py -q --timeout 200 --timeout-method thread > gpurun_out/ab/$n.log 2>&1
  echo "$n: $(tail -1 gpurun_out/ab/$n.log)"
  grep -E "^E +AssertionError" gpurun_out/ab/$n.log | head -5
done
bash scripts/ab_libs.sh
