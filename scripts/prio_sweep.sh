#!/bin/bash
# NUTS-wave priority experiment: short headline-shape runs at each s_setprio level.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prio
for c in 3 5 2; do
  for p in 3 1 0; do
    FITOCT_NUTS_PRIO=$p timeout -k 10 200 python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu --iters 200,200 > gpurun_out/prio/c${c}_p$p.json 2>gpurun_out/prio/err || { tail gpurun_out/prio/err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/prio/c${c}_p$p.json'));print('config $c prio $p', d['value'], d['roofline']['kernel_ms'])"
  done
done
