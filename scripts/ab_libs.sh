#!/bin/bash
# A/B: every abtest/lib_*.so on configs 3, 4, 2, 5 (short runs), interleaved twice.
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for c in ${AB_CONFIGS:-3 4 2 5}; do
    for l in abtest/lib_*.so; do
      it="200,200"; [ $c = 5 ] && it="100,100"
      FITOCT_LIB_PATH=$PWD/$l timeout -k 10 150 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --iters $it 2>>gpurun_out/ab_stderr.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$l config $c', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'])" || exit 1
    done
  done
done
