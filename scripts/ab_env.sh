#!/bin/bash
# Runtime-switch A/B on configs 2 and 5 (short runs): default vs FITOCT_NO_MIGRATE=1.
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for c in ${AB_CONFIGS:-2 5}; do
    for envs in "X=0" "FITOCT_NO_MIGRATE=1"; do
      it="200,200"; [ $c = 5 ] && it="100,100"
      env $envs timeout -k 10 150 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --iters $it 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$envs config $c', d['value'], d['roofline']['kernel_ms'])" || exit 1
    done
  done
done
