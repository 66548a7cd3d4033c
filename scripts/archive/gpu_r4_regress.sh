#!/bin/bash
# Round 4: regression check of the round-4 library against the round-3 final tree (1c4bc43,
# built in abtest/r3 with its own bench.py), config 3 full length, interleaved twice on one
# box; plus config 2 and 5 short runs.  Outputs gpurun_out/r4reg/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4reg
mkdir -p $OUT
run() {   # name dir args
  (cd $2 && timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err) | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" >> $OUT/ab.txt
}
for rep in 1 2; do
  run r4 $GRAFT_REPO_ROOT "--steps 1 --warmup 0" || exit 1
  run r3 $GRAFT_REPO_ROOT/abtest/r3 "--steps 1 --warmup 0" || exit 1
done
for rep in 1 2; do
  for c in 2 5; do
    run r4 $GRAFT_REPO_ROOT "--config $c --steps 2 --warmup 1" || exit 1
    run r3 $GRAFT_REPO_ROOT/abtest/r3 "--config $c --steps 2 --warmup 1" || exit 1
  done
done
cat $OUT/ab.txt
