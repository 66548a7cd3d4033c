#!/bin/bash
# Round 4: priorities of the chain wave's in-sweep prior part and of the helper wave in one-chain
# tiles with deep speculation (config 2), FITOCT_DEEP_PRIOR_PRIO / FITOCT_HELPER_PRIO variants in
# abtest/lib_*.so against the main library; 4 steps each, interleaved twice.  Outputs gpurun_out/r4prio/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4prio
mkdir -p $OUT
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'frac', d['roofline']['frac'])" >> $OUT/ab.txt
}
for rep in 1 2; do
  run main "FITOCT_NOP=1" "--config 2 --steps 4 --warmup 1" || exit 1
  for v in ${VARIANTS:-prior0 helper0 both0 helper2}; do
    run $v "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_$v.so" "--config 2 --steps 4 --warmup 1" || exit 1
  done
done
cat $OUT/ab.txt
