#!/bin/bash
# A/B: config 5 (and a short config 3) with libraries built at earlier commits (abtest/).
cd "$GRAFT_REPO_ROOT"
for l in abtest/lib_*.so; do
  for c in 5 2 3; do
    it="100,100"; [ $c != 5 ] && it="200,200"
    FITOCT_LIB_PATH=$PWD/$l timeout -k 10 150 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu --iters $it 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$l config $c', d['value'], d['roofline']['kernel_ms'])"
  done
done
