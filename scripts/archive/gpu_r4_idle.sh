#!/bin/bash
# Round 4: the chain wave's idle wait during a two-ended tree: main (NUTS priority, s_sleep 1)
# vs idle8 (s_sleep 8) vs idle0 (priority 0, s_sleep 8), config 2, 4 steps each, interleaved twice.
# Outputs gpurun_out/r4idle/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4idle
mkdir -p $OUT
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'R-hat', d.get('rhat_max'))" >> $OUT/ab.txt
}
for rep in 1 2; do
  run main "FITOCT_NOP=1" "--config 2 --steps 4 --warmup 1" || exit 1
  run idle8 "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_idle8.so" "--config 2 --steps 4 --warmup 1" || exit 1
  run idle0 "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_idle0.so" "--config 2 --steps 4 --warmup 1" || exit 1
done
cat $OUT/ab.txt
