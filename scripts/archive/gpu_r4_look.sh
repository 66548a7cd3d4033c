#!/bin/bash
# Round 4: two-ended trajectories' lookahead (FITOCT_BIDI_LOOK 1 = main, 2, 3) and a short ring
# (FITOCT_BIDI_RB=16), config 2, 4 steps each, interleaved twice.  Outputs gpurun_out/r4look/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4look
mkdir -p $OUT
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'R-hat', d.get('rhat_max'))" >> $OUT/ab.txt
}
for rep in 1 2; do
  run look1 "FITOCT_NOP=1" "--config 2 --steps 4 --warmup 1" || exit 1
  run look2 "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_look2.so" "--config 2 --steps 4 --warmup 1" || exit 1
  run look3 "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_look3.so" "--config 2 --steps 4 --warmup 1" || exit 1
  run rb16 "FITOCT_BIDI_RB=16" "--config 2 --steps 4 --warmup 1" || exit 1
done
cat $OUT/ab.txt
