#!/bin/bash
# Secondary bench lines: BASELINE.json configs 2 and 4 (one step each, no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/configs
for c in ${CONFIGS:-2 4}; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu > gpurun_out/configs/c$c.json 2> gpurun_out/configs/c$c.err || { echo "config $c failed"; tail -20 gpurun_out/configs/c$c.err; exit 1; }
  cat gpurun_out/configs/c$c.json
done
