#!/bin/bash
# Round 4: A/B of the lagging-wave priority (FITOCT_LAG_PRIO = 0 off, 1, 2, 3) on config 3,
# short runs (200 + 200) interleaved twice, then full length for 0 and the short-run best.
# Outputs gpurun_out/r4lag/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4lag
mkdir -p $OUT
run() {   # name env iters steps
  env $2 timeout -k 10 300 python3 bench.py --steps $4 --warmup 1 --no-cpu --no-hard --iters $3 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'stuck', d['stuck_chains'])" >> $OUT/ab.txt
}
for rep in 1 2; do
  for l in 0 1 2 3; do run lag$l "FITOCT_LAG_PRIO=$l" 200,200 2 || exit 1; done
done
cat $OUT/ab.txt
for rep in 1 2; do
  for l in 0 1 2 3; do run lag$l "FITOCT_LAG_PRIO=$l" 500,1000 1 || exit 1; done
done
cat $OUT/ab.txt
