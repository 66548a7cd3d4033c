#!/bin/bash
# Round 4: locate the config-3 regression against the round-3 tree (abtest/r3): round-4 library,
# variants without the timeout-NaN outputs (lib_nonan) and with KParams.theta_rate moved to
# the end of the struct (lib_ratelast), interleaved twice, full length, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4reg2
mkdir -p $OUT
run() {   # name dir env
  (cd $2 && env $3 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard 2>>$OUT/ab.err) | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'grads', d['roofline']['gradients_per_launch'])" >> $OUT/ab.txt
}
for rep in 1 2; do
  run r4 $GRAFT_REPO_ROOT "FITOCT_NOP=1" || exit 1
  run nonan $GRAFT_REPO_ROOT "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_nonan.so" || exit 1
  run ratelast $GRAFT_REPO_ROOT "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_ratelast.so" || exit 1
  run r3 $GRAFT_REPO_ROOT/abtest/r3 "FITOCT_NOP=1" || exit 1
done
cat $OUT/ab.txt
